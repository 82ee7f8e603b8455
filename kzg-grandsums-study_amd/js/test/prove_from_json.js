// Test driver used by tests/test_js_dropin.py: read {ptau, cases:[{kind, F:[hex], T:[hex], selF, selT}]}
// from argv[2], run the drop-in provers, print {proofs:[{commitments:{k:hex}, evaluations:{k:hex}, montF:[hex]}]}.
// With spec.concurrent every case is started at once (Promise.all), as independent reference calls
// would be (src/grandsum/mset_eq_kzg_prover.js:12 is an independent async function per call). A case
// with replacePtau first copies that file over spec.ptau (a ptau rewritten between two calls).
const fs = require("fs");
const { getCurveFromName, Evaluations, mset_eq_kzg_grandsum_prover, mset_eq_kzg_grandproduct_prover,
        lookup_kzg_grandsum_prover, mset_eq_kzg_grandsum_verifier, mset_eq_kzg_grandproduct_verifier,
        lookup_kzg_grandsum_verifier } = require("../index");

(async () => {
    const spec = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));
    const curve = await getCurveFromName("bn128");
    const hex = b => Buffer.from(b).toString("hex");
    const ev = h => new Evaluations(new Uint8Array(Buffer.from(h, "hex")), curve);
    const one = async c => {
        if (c.replacePtau) fs.copyFileSync(c.replacePtau, spec.ptau);
        const F = c.F.map(ev), T = c.T.map(ev);
        const fn = { grandsum: mset_eq_kzg_grandsum_prover, grandproduct: mset_eq_kzg_grandproduct_prover,
                     lookup: lookup_kzg_grandsum_prover }[c.kind];
        try {
            const proof = await fn(spec.ptau, F.length === 1 ? F[0] : F, T.length === 1 ? T[0] : T,
                c.selF ? ev(c.selF) : null, c.selT ? ev(c.selT) : null);
            const o = { commitments: {}, evaluations: {}, montF: F.map(e => hex(e.eval)) };
            for (const k of Object.keys(proof.commitments)) o.commitments[k] = hex(proof.commitments[k]);
            for (const k of Object.keys(proof.evaluations)) o.evaluations[k] = hex(proof.evaluations[k]);
            if (spec.verify) {  // the drop-in verifier of the same argument, as the reference's tests do
                const vf = { grandsum: mset_eq_kzg_grandsum_verifier, grandproduct: mset_eq_kzg_grandproduct_verifier,
                             lookup: lookup_kzg_grandsum_verifier }[c.kind];
                o.verified = await vf(spec.ptau, proof, Math.log2(F[0].length()));
            }
            return o;
        } catch (e) {
            return { error: e.message, errorName: e.name };
        }
    };
    let out;
    if (spec.concurrent) {
        out = await Promise.all(spec.cases.map(one));
    } else {
        out = [];
        for (const c of spec.cases) out.push(await one(c));
    }
    const { poolInfo } = require("../src/backend");
    console.log(JSON.stringify({ proofs: out, pool: poolInfo() }));
})().catch(e => { console.error(e); process.exit(1); });
