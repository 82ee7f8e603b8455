// Test driver used by tests/test_js_verifier_log.py (CPU: the verifier is host-only, no GPU call):
// read {ptau, cases:[{kind, nbits, proof:{commitments:{k:hex}, evaluations:{k:hex}}, drop?}]} from
// argv[2], run the drop-in verifier module of each case's kind with a capturing logger, print
// {cases:[{valid, lines:[...], threw}]} ("I " / "E " prefix = logger.info / logger.error).
const fs = require("fs");
const logger = require("../src/logger");
const MOD = {
    grandsum: require("../src/grandsum/mset_eq_kzg_verifier"),
    grandproduct: require("../src/grandproduct/mset_eq_kzg_verifier"),
    lookup: require("../src/lookup/lookup_kzg_verifier"),
};

(async () => {
    const spec = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));
    const u8 = h => new Uint8Array(Buffer.from(h, "hex"));
    const out = [];
    for (const c of spec.cases) {
        const lines = [];
        logger.setLogger({ info: (...a) => lines.push("I " + a.join(" ")), error: (...a) => lines.push("E " + a.join(" ")) });
        const proof = { commitments: {}, evaluations: {} };
        for (const k of Object.keys(c.proof.commitments)) proof.commitments[k] = u8(c.proof.commitments[k]);
        for (const k of Object.keys(c.proof.evaluations)) proof.evaluations[k] = u8(c.proof.evaluations[k]);
        if (c.drop) delete proof[c.drop[0]][c.drop[1]];
        let valid = null, threw = null;
        try {
            valid = await MOD[c.kind](spec.ptau, proof, c.nbits);
        } catch (e) {
            threw = e.message;
        }
        out.push({ valid, lines, threw });
    }
    logger.setLogger(null);
    console.log(JSON.stringify({ cases: out }));
})().catch(e => { console.error(e); process.exit(1); });
