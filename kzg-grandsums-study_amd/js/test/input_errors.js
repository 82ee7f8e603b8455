// Test driver used by tests/test_input_errors.py: the drop-in provers' input checks
// (src/grandsum/mset_eq_kzg_prover.js:22-81, same in the grand-product prover) run before any GPU
// work, so this needs no device. Prints {kind: [message per case]} as JSON.
const { getCurveFromName, Evaluations, mset_eq_kzg_grandsum_prover, mset_eq_kzg_grandproduct_prover,
        lookup_kzg_grandsum_prover } = require("../index");

(async () => {
    const ptau = process.argv[2];  // a small ptau (power < 8)
    const curve = await getCurveFromName("bn128");
    const ev = n => Evaluations.getRandomEvals(n, curve);
    const one = n => Evaluations.getOneEvals(n, curve);
    const cases = [
        () => [[ev(8), ev(8)], [ev(8)], null, null],      // vector lengths differ
        () => [[], [], null, null],                       // no multisets
        () => [ev(8), ev(4), null, null],                 // 0-th buffers differ
        () => [[ev(8), ev(4)], [ev(8), ev(4)], null, null],  // multisets of different lengths
        () => [ev(8), ev(8), one(8), one(4)],             // selection buffers differ
        () => [ev(8), ev(8), one(4), one(4)],             // selection vs multiset length
        () => [ev(6), ev(6), null, null],                 // not a power of two
        () => [ev(256), ev(256), null, null],             // ptau too small
    ];
    const out = {};
    for (const [kind, fn] of [["grandsum", mset_eq_kzg_grandsum_prover], ["grandproduct", mset_eq_kzg_grandproduct_prover],
                              ["lookup", lookup_kzg_grandsum_prover]]) {
        out[kind] = [];
        for (const mk of cases) {
            const [F, T, sF, sT] = mk();
            try {
                await fn(ptau, F, T, sF, kind === "lookup" && sT === null ? one(Array.isArray(F) ? (F[0] ? F[0].length() : 8) : F.length()) : sT);
                out[kind].push("no error");
            } catch (e) {
                out[kind].push(e.message);
            }
        }
    }
    console.log(JSON.stringify(out));
    process.exit(0);
})().catch(e => { console.error(e); process.exit(1); });
