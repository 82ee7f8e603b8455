// The reference's own test cases (test/mset_eq_kzg_grandsum.test.js:24-104 and the grand-product
// twin) driven through the drop-in modules, without mocha: random inputs via curve.Fr.random, T = F
// rotated by one, selectors ones except selF[n-1] = selT[0] = 0. Like the reference's tests, every
// proof must pass the verifier (here the drop-in verifier module: native transcript replay + pairing).
// Plus the "standard lookup" of test/lookup_kzg_grandsum.test.js:24-44 (commented out in the
// reference) through the lookup modules: it verifies there, and the grand-sum prover refuses it.
const path = require("path");
const { getCurveFromName, Evaluations, mset_eq_kzg_grandsum_prover, mset_eq_kzg_grandproduct_prover,
    mset_eq_kzg_grandsum_verifier, mset_eq_kzg_grandproduct_verifier, lookup_kzg_grandsum_prover,
    lookup_kzg_grandsum_verifier } = require("../index");

async function main() {
    const ptau = process.argv[2] || path.join("tmp", "powersOfTau28_hez_final_11.ptau");
    const curve = await getCurveFromName("bn128");
    const Fr = curve.Fr;
    let pass = 0;
    for (const [name, fn, sname, vf] of [["grandsum", mset_eq_kzg_grandsum_prover, "S", mset_eq_kzg_grandsum_verifier],
                                         ["grandproduct", mset_eq_kzg_grandproduct_prover, "Z", mset_eq_kzg_grandproduct_verifier]]) {
        for (const [nPols, sel] of [[1, false], [3, false], [1, true], [2, true]]) {
            const nBits = 1 + Math.floor(Math.random() * 6);
            const mk = () => {
                const evalsF = Evaluations.getRandomEvals(2 ** nBits, curve);
                const evalsT = Evaluations.fromEvals(evalsF);
                evalsT.setEvaluation(1, evalsF.getEvaluationSequence(0, evalsF.length() - 1));
                evalsT.setEvaluation(0, evalsF.getEvaluation(evalsF.length() - 1));
                return [evalsF, evalsT];
            };
            const Fs = [], Ts = [];
            for (let i = 0; i < nPols; i++) { const [f, t] = mk(); Fs.push(f); Ts.push(t); }
            let sF = null, sT = null;
            if (sel) {
                sF = Evaluations.getOneEvals(2 ** nBits, curve);
                sT = Evaluations.fromEvals(sF);
                sF.setEvaluation(sF.length() - 1, Fr.zero);
                sT.setEvaluation(0, Fr.zero);
            }
            const proof = await fn(ptau, nPols === 1 ? Fs[0] : Fs, nPols === 1 ? Ts[0] : Ts, sF, sT);
            const keys = Object.keys(proof.commitments);
            if (!keys.includes(sname) || !keys.includes("Q") || !keys.includes("Wxi") || !keys.includes("Wxiw"))
                throw new Error(`${name}: bad proof keys ${keys}`);
            if (sel !== keys.includes("selF")) throw new Error("selector commitments mismatch");
            const isValid = await vf(ptau, proof, nBits);  // test/mset_eq_kzg_grandsum.test.js: assert(isValid)
            if (isValid !== true) throw new Error(`${name} nPols=${nPols} sel=${sel} nBits=${nBits}: proof rejected`);
            pass++;
        }
    }
    {
        // test/lookup_kzg_grandsum.test.js:25-43: F = T with F[1] = F[n-1] = F[0]; multiplicities ones
        // except m[0] = 3, m[1] = m[n-1] = 0
        const nBits = 2;
        const evalsT = Evaluations.getRandomEvals(2 ** nBits, curve);
        const evalsF = Evaluations.fromEvals(evalsT);
        evalsF.setEvaluation(1, evalsF.getEvaluation(0));
        evalsF.setEvaluation(evalsF.length() - 1, evalsF.getEvaluation(0));
        const mul = Evaluations.getOneEvals(2 ** nBits, curve);
        mul.setEvaluation(0, Fr.e(3));
        mul.setEvaluation(1, Fr.zero);
        mul.setEvaluation(mul.length() - 1, Fr.zero);
        const copy = e => Evaluations.fromEvals(e);
        const proof = await lookup_kzg_grandsum_prover(ptau, copy(evalsF), copy(evalsT),
            Evaluations.getOneEvals(2 ** nBits, curve), copy(mul));
        if ((await lookup_kzg_grandsum_verifier(ptau, proof, nBits)) !== true) throw new Error("lookup proof rejected");
        pass++;
        let refused = false;
        try {
            await mset_eq_kzg_grandsum_prover(ptau, copy(evalsF), copy(evalsT), Evaluations.getOneEvals(2 ** nBits, curve), copy(mul));
        } catch (e) {
            refused = e.message === "Polynomial is not divisible";
        }
        if (!refused) throw new Error("the grand-sum prover accepted multiplicities");
        pass++;
    }
    console.log(`reference-style cases passed: ${pass}`);
}
main().catch(e => { console.error(e); process.exit(1); });
