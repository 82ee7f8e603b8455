// Device backend: one libkgs context per HIP device, device-resident SRS cached per ptau path.
const path = require("path");

let addon = null;
function load() {
    if (!addon) {
        const p = process.env.KGS_ADDON || path.join(__dirname, "..", "build", "kgs_addon.node");
        addon = require(p);  // no CPU fallback: the HIP library is the only path
    }
    return addon;
}

const contexts = new Map();
const loaded = new Map();

async function context(device = 0) {
    const a = load();
    if (!contexts.has(device)) contexts.set(device, a.ctxCreate(device));
    return contexts.get(device);
}

async function loadPtau(ctx, pTauFilename) {
    const key = path.resolve(pTauFilename);
    if (loaded.get(ctx) !== key) {
        await load().srsLoadPtau(ctx, key, -1);
        loaded.set(ctx, key);
    }
    return load().srsInfo(ctx);
}

async function prove(kind, pTauFilename, nBits, evalsF, evalsT, selF, selT, device = 0) {
    const ctx = await context(device);
    await loadPtau(ctx, pTauFilename);
    return load().prove(ctx, kind, nBits, evalsF, evalsT, selF, selT);
}

module.exports = { load, context, loadPtau, prove, GRANDSUM: 0, GRANDPRODUCT: 1 };
