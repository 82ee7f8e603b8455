// Test driver used by tests/test_js_dropin.py: read {ptau, cases:[{kind, F:[hex], T:[hex], selF, selT}]}
// from argv[2], run the drop-in provers, print {proofs:[{commitments:{k:hex}, evaluations:{k:hex}, montF:[hex]}]}.
const fs = require("fs");
const { getCurveFromName, Evaluations, mset_eq_kzg_grandsum_prover, mset_eq_kzg_grandproduct_prover } = require("../index");

(async () => {
    const spec = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));
    const curve = await getCurveFromName("bn128");
    const hex = b => Buffer.from(b).toString("hex");
    const ev = h => new Evaluations(new Uint8Array(Buffer.from(h, "hex")), curve);
    const out = [];
    for (const c of spec.cases) {
        const F = c.F.map(ev), T = c.T.map(ev);
        const fn = c.kind === "grandsum" ? mset_eq_kzg_grandsum_prover : mset_eq_kzg_grandproduct_prover;
        try {
            const proof = await fn(spec.ptau, F.length === 1 ? F[0] : F, T.length === 1 ? T[0] : T,
                c.selF ? ev(c.selF) : null, c.selT ? ev(c.selT) : null);
            const o = { commitments: {}, evaluations: {}, montF: F.map(e => hex(e.eval)) };
            for (const k of Object.keys(proof.commitments)) o.commitments[k] = hex(proof.commitments[k]);
            for (const k of Object.keys(proof.evaluations)) o.evaluations[k] = hex(proof.evaluations[k]);
            out.push(o);
        } catch (e) {
            out.push({ error: e.message });
        }
    }
    console.log(JSON.stringify({ proofs: out }));
})().catch(e => { console.error(e); process.exit(1); });
