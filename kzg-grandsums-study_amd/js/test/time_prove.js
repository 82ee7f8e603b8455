// Times the JavaScript drop-in prover end to end (module call -> N-API -> libkgs -> proof object),
// as a reference user would call it: node time_prove.js PTAU NBITS [PROOFS]. Inputs are random
// standard-form field elements (< 2^253 < r) in Uint8Arrays, T = F rotated by one element.
// Prints one JSON line: {nbits, proofs, ms_per_proof, proofs_per_s, verified}.
const crypto = require("crypto");
const { getCurveFromName, Evaluations, mset_eq_kzg_grandsum_prover, mset_eq_kzg_grandsum_verifier } = require("../index");

(async () => {
    const [ptau, nbArg, nArg] = process.argv.slice(2);
    const nBits = parseInt(nbArg, 10), proofs = parseInt(nArg || "5", 10);
    const n = 2 ** nBits;
    const curve = await getCurveFromName("bn128");
    const f = new Uint8Array(crypto.randomBytes(32 * n));
    for (let i = 0; i < n; i++) f[32 * i + 31] &= 0x1f;  // < 2^253
    const t = new Uint8Array(32 * n);
    t.set(f.subarray(0, 32 * (n - 1)), 32);
    t.set(f.subarray(32 * (n - 1)), 0);
    const mk = () => [new Evaluations(f.slice(), curve), new Evaluations(t.slice(), curve)];
    let [F, T] = mk();
    let proof = await mset_eq_kzg_grandsum_prover(ptau, F, T);  // warm: context, SRS, buffers
    let best = Infinity;
    for (let i = 0; i < proofs; i++) {
        [F, T] = mk();  // fresh standard-form inputs (the prover overwrites them with Montgomery form)
        const t0 = process.hrtime.bigint();
        proof = await mset_eq_kzg_grandsum_prover(ptau, F, T);
        const ms = Number(process.hrtime.bigint() - t0) / 1e6;
        best = Math.min(best, ms);
    }
    const verified = await mset_eq_kzg_grandsum_verifier(ptau, proof, nBits);
    console.log(JSON.stringify({ nbits: nBits, proofs, ms_per_proof: +best.toFixed(3), proofs_per_s: +(1000 / best).toFixed(3), verified }));
    process.exit(0);
})().catch(e => { console.error(e); process.exit(1); });
