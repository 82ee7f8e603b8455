// Test driver used by tests/test_verifier.py: read {ptau, cases:[{kind, nbits, commitments:{k:hex},
// evaluations:{k:hex}}]} from argv[2], run the drop-in verifiers, print {verdicts:[bool|string]}.
const fs = require("fs");
const { mset_eq_kzg_grandsum_verifier, mset_eq_kzg_grandproduct_verifier, lookup_kzg_grandsum_verifier } = require("../index");

(async () => {
    const spec = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));
    const u8 = h => new Uint8Array(Buffer.from(h, "hex"));
    const out = [];
    for (const c of spec.cases) {
        const proof = { commitments: {}, evaluations: {} };
        for (const k of Object.keys(c.commitments)) proof.commitments[k] = u8(c.commitments[k]);
        for (const k of Object.keys(c.evaluations)) proof.evaluations[k] = u8(c.evaluations[k]);
        const fn = { grandsum: mset_eq_kzg_grandsum_verifier, grandproduct: mset_eq_kzg_grandproduct_verifier,
                     lookup: lookup_kzg_grandsum_verifier }[c.kind];
        try {
            out.push(await fn(spec.ptau, proof, c.nbits));
        } catch (e) {
            out.push(e.message);
        }
    }
    console.log(JSON.stringify({ verdicts: out }));
})().catch(e => { console.error(e); process.exit(1); });
