// Test driver used by tests/test_js_log.py (CPU: no GPU call): read {cases:[{kind, nbits, npols,
// selected, proof:{commitments:{k:hex}, evaluations:{k:hex}}}]} from argv[2], replay each proof's
// transcript through the drop-in prover's round log (prover_common.logRounds, the reference's log
// lines) into a capturing logger, print {cases:[{challenges:{name:decimal}, lines:[...]}]}.
const fs = require("fs");
const logger = require("../src/logger");
const { logRounds } = require("../src/prover_common");
const { getCurveFromName } = require("../src/curve");

(async () => {
    const spec = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));
    const curve = await getCurveFromName("bn128");
    const kinds = { grandsum: 0, grandproduct: 1, lookup: 2 };
    const u8 = h => new Uint8Array(Buffer.from(h, "hex"));
    const out = [];
    for (const c of spec.cases) {
        const lines = [];
        logger.setLogger({ info: (...a) => lines.push(a.join(" ")), warn: (...a) => lines.push("WARN " + a.join(" ")) });
        const proof = { commitments: {}, evaluations: {} };
        for (const k of Object.keys(c.proof.commitments)) proof.commitments[k] = u8(c.proof.commitments[k]);
        for (const k of Object.keys(c.proof.evaluations)) proof.evaluations[k] = u8(c.proof.evaluations[k]);
        const ch = logRounds(kinds[c.kind], curve, proof, c.nbits, c.npols, c.selected);
        const challenges = {};
        for (const k of Object.keys(ch)) if (ch[k] !== null) challenges[k] = curve.Fr.toString(ch[k]);
        out.push({ challenges, lines });
    }
    logger.setLogger(null);
    console.log(JSON.stringify({ cases: out }));
})().catch(e => { console.error(e); process.exit(1); });
