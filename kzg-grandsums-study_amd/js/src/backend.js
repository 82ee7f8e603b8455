// Device backend: a pool of libkgs contexts spread over the visible HIP devices.
//
// The reference prover is an independent async function per call
// (src/grandsum/mset_eq_kzg_prover.js:12): `Promise.all([prover(a), prover(b)])` runs both. Here
// every call takes a context slot for its whole duration (SRS load + prove), so a context is never
// used by two calls at once, and independent calls run concurrently on different contexts (each
// with its own HIP stream and buffers, on the same GPU or on another one). libkgs additionally
// serialises calls per context with a mutex, and shares the read-only SRS / NTT tables between the
// contexts of a device, so a pool of several contexts costs one set of tables per GPU.
//
// Knobs: KGS_JS_CONTEXTS = contexts per device (default 8: with 16 concurrent calls, 8 contexts
// reach 82 proofs/s at n = 2^20 against 78.5 with 4, profiles/r02/js_adaptive_lanes.txt), KGS_DEVICES = comma-separated device list (default: every visible device),
// KGS_JS_SHARD_RANKS / KGS_JS_SHARD_MIN_NBITS = one large proof over several GPUs (below).
const fs = require("fs");
const path = require("path");
const { contiguous } = require("./bigbuffer");

// N-API async work runs on the libuv thread pool (4 threads by default): one thread per context of
// an 8-GPU pool needs more. Effective only if set before the process first uses the pool.
if (!process.env.UV_THREADPOOL_SIZE) process.env.UV_THREADPOOL_SIZE = "64";

let addon = null;
function load() {
    if (!addon) {
        const p = process.env.KGS_ADDON || path.join(__dirname, "..", "build", "kgs_addon.node");
        addon = require(p);  // no CPU fallback: the HIP library is the only path
    }
    return addon;
}

function devices() {
    const env = process.env.KGS_DEVICES;
    if (env && env.trim() !== "") return env.split(",").map(x => parseInt(x, 10)).filter(x => x >= 0);
    const n = load().deviceCount();
    if (n < 1) throw new Error("no HIP device visible");
    return Array.from({ length: n }, (_, i) => i);
}

function perDevice() {
    const v = parseInt(process.env.KGS_JS_CONTEXTS || "8", 10);
    return Number.isFinite(v) && v >= 1 ? v : 8;
}

const pool = { slots: [], idle: [], waiters: [], devs: null, cap: 0 };
const diag = { execMs: null, timing: null, waitMs: null, callMs: null };

function newSlot() {
    if (!pool.devs) {
        pool.devs = devices();
        pool.cap = pool.devs.length * perDevice();
    }
    // round-robin over devices: slot i lives on device devs[i % ndev]
    const device = pool.devs[pool.slots.length % pool.devs.length];
    const slot = { device, ctx: load().ctxCreate(device), index: pool.slots.length, busy: false, lanes: 2 };
    pool.slots.push(slot);
    return slot;
}

function acquire() {
    if (pool.idle.length) return Promise.resolve(pool.idle.pop());
    if (!pool.devs || pool.slots.length < pool.cap) return Promise.resolve(newSlot());
    return new Promise(resolve => pool.waiters.push(resolve));
}

function release(slot) {
    const w = pool.waiters.shift();
    if (w) w(slot);
    else pool.idle.push(slot);
}

// run fn(slot) with exclusive use of one context
async function withContext(fn) {
    const slot = await acquire();
    slot.busy = true;
    try {
        return await fn(slot);
    } finally {
        slot.busy = false;
        release(slot);
    }
}

// Eager collection beside a lone proof: OPT-IN (KGS_JS_EAGER_GC=1, or =<ms> for the delay), and only
// in an application that itself started Node with --expose-gc (the library never changes V8 flags).
// Why it exists: every proof leaves the caller's previous input buffers (the reference replaces
// Evaluations.eval by the Montgomery copy, prover.js:147-148) as 64 MiB of garbage at n = 2^20; V8
// then finalises a ~6 ms mark-sweep as a main-thread task, which, scheduled while the GPU works, tended
// to run just as the proof completed: the Promise resolved 0.1-5 ms after the result was ready
// (profiles/r04/js/). With the opt-in, a proof alone on its device runs one full collection
// GC_DELAY_MS after it is queued, beside its ~15 ms of GPU work (not at once: freeing the garbage's
// pages while round 1 copies the next inputs into pinned staging stretched that round from 3.4 to
// 9-15 ms in a third of the samples, profiles/r04/js/run5); with other proofs in flight V8's own
// schedule is kept. A blocking full collection on the host application's main thread is its call to
// make, which is why this is off by default.
const GC_DELAY_MS = (() => {
    const v = parseInt(process.env.KGS_JS_EAGER_GC || "", 10);
    return Number.isFinite(v) && v > 1 ? v : 5;
})();
function eagerGcEnabled() {
    const v = process.env.KGS_JS_EAGER_GC;
    return v !== undefined && v !== "" && v !== "0" && typeof global.gc === "function";
}
// Only proofs whose inputs are large enough for their garbage to matter (>= 16 MiB of F / T, e.g.
// n >= 2^18 for one pair) schedule it, and at most one collection is pending at a time: small proofs
// take less than the collection itself.
const GC_MIN_BYTES = 16 << 20;
let gcPending = false;
function scheduleCollect(inputBytes) {
    if (!eagerGcEnabled() || gcPending || inputBytes < GC_MIN_BYTES) return;
    gcPending = true;
    setTimeout(() => {
        gcPending = false;
        global.gc();
    }, GC_DELAY_MS);
}

// MSM lanes of a proof about to start: two (single-proof latency mode, kgs_ctx_set_msm_lanes) when it
// is alone on its device, one when other proofs are in flight there or waiting for a context — the
// GPU is then already full, and the two-lane accumulation's register reservation would keep the
// other contexts' kernels from co-residing (DESIGN.md §3 register budget)
function setLanes(slot) {
    const others = pool.slots.some(s => s !== slot && s.busy && s.device === slot.device);
    const lanes = others || pool.waiters.length > 0 ? 1 : 2;
    if (slot.lanes !== lanes) {
        load().ctxSetMsmLanes(slot.ctx, lanes);
        slot.lanes = lanes;
    }
}

// ptau header power, read without a context (readPTauHeader, src/ptau_utils.js:3-24)
function ptauPower(pTauFilename) {
    return load().ptauPower(path.resolve(pTauFilename));
}

// SRS load (only 2^(nBits+1) points, as prover.js:83-85 reads; grow-only device cache in libkgs)
// and prove on the same held context: nothing can swap the SRS between the two
async function prove(kind, pTauFilename, nBits, evalsF, evalsT, selF, selT) {
    const key = path.resolve(pTauFilename);
    // evaluations held in a BigBuffer (Evaluations.fromPolynomial, src/polynomial/evaluations.js:12-21)
    // go to the native side as one contiguous copy
    evalsF = evalsF.map(contiguous);
    evalsT = evalsT.map(contiguous);
    if (selF) selF = contiguous(selF);
    if (selT) selT = contiguous(selT);
    if (shardRanks() >= 2 && nBits >= shardMinBits()) return proveSharded(kind, key, nBits, evalsF, evalsT, selF, selT);
    return withContext(async slot => {
        // the SRS load is an async job (a libuv thread round trip) even when libkgs finds its tables
        // already resident; skip it when this context loaded the same file (same real path, size and
        // mtime — the identity libkgs checks, so a rewritten ptau is still re-read) for >= nBits
        // (a file that cannot be stat'ed goes to libkgs, which reports it as the drop-in always has)
        let id = null;
        try {
            const st = fs.statSync(key, { bigint: true });
            id = `${fs.realpathSync(key)}#${st.size}#${st.mtimeNs}`;
        } catch (e) {
            id = null;
        }
        if (id === null || slot.srsId !== id || slot.srsBits < nBits) {
            slot.srsId = null;
            await load().srsLoadPtau(slot.ctx, key, nBits);
            slot.srsId = id;
            slot.srsBits = nBits;
        }
        setLanes(slot);
        const t0 = process.hrtime.bigint();
        const pending = load().prove(slot.ctx, kind, nBits, evalsF, evalsT, selF, selT);
        if (slot.lanes === 2) {  // alone on its device: see scheduleCollect (opt-in)
            scheduleCollect(evalsF.concat(evalsT).reduce((a, e) => a + e.length, 0));
        }
        const res = await pending;
        // diagnostics of the last call: the native call's wall time, its [queue -> worker, worker ->
        // completion] waits, time inside libkgs, kgs_last_timing rounds / copy / prover / write-back
        diag.callMs = Number(process.hrtime.bigint() - t0) / 1e6;
        diag.waitMs = res.waitMs;
        diag.execMs = res.execMs;
        diag.timing = load().lastTiming(slot.ctx);
        return res;
    });
}

// Large proofs over several GPUs from this one Node process: with KGS_JS_SHARD_RANKS = W >= 2, a
// proof of at least 2^KGS_JS_SHARD_MIN_NBITS elements (default 22) runs on W contexts (rank r on
// device r mod #devices) joined by an in-process rank group (kgs_group_create_local +
// kgs_ctx_set_group): every vector of the proof sharded, NTTs as rank-local transforms plus one
// all-to-all, every MSM over the rank's slice of the SRS, which is all a rank loads
// (kgs_srs_load_ptau_slice; DESIGN.md §6). The W ranks run as ONE async job that starts one native
// thread per rank (addon proveGroup), so they never wait for libuv pool threads held by other work;
// rank 0 returns the proof and the Montgomery write-back. One sharded proof at a time (the group's
// barriers join the ranks of one proof); the same inputs and the same Promise result as the
// single-GPU path.
const shard = { ctxs: null, group: null, busy: Promise.resolve() };
function shardRanks() {
    const v = parseInt(process.env.KGS_JS_SHARD_RANKS || "0", 10);
    return Number.isFinite(v) ? v : 0;
}
function shardMinBits() {
    const v = parseInt(process.env.KGS_JS_SHARD_MIN_NBITS || "22", 10);
    return Number.isFinite(v) ? v : 22;
}
function proveSharded(kind, key, nBits, evalsF, evalsT, selF, selT) {
    const a = load();
    const W = shardRanks();
    const run = async () => {
        if (!shard.ctxs || shard.ctxs.length !== W) {
            const devs = devices();
            shard.ctxs = Array.from({ length: W }, (_, r) => a.ctxCreate(devs[r % devs.length]));
            shard.group = null;
        }
        if (!shard.group) {
            shard.group = a.groupCreateLocal(W);
            shard.ctxs.forEach((c, r) => a.ctxSetGroup(c, shard.group, r));
        }
        try {
            return await a.proveGroup(shard.ctxs, key, kind, nBits, evalsF, evalsT, selF, selT);
        } catch (e) {
            // a rank failed: the group may be spent (the others were released with an error); make a
            // fresh one for the next proof
            shard.ctxs.forEach(c => a.ctxSetGroup(c, null, 0));
            shard.group = null;
            throw e;
        }
    };
    const p = shard.busy.then(run, run);
    shard.busy = p.catch(() => {});
    return p;
}

function poolInfo() {
    return { contexts: pool.slots.length, capacity: pool.cap, devices: pool.devs ? pool.devs.slice() : null,
             idle: pool.idle.length, waiting: pool.waiters.length };
}

module.exports = { load, ptauPower, prove, withContext, poolInfo, diag, GRANDSUM: 0, GRANDPRODUCT: 1, LOOKUP: 2 };
