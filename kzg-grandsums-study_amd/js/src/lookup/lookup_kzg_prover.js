// Lookup prover (SURVEY.md §8f N4). The reference's lookup tests (test/lookup_kzg_grandsum.test.js:24-44,
// commented out) call the grand-sum prover with (F, T, selF, multiplicities); this module is that call
// with the multiplicities' binary constraint dropped (include/kgs.h KGS_LOOKUP): every selected row of
// F must be a row of T, evalsMulT[j] counting how often row j is looked up. Same arguments, Promise
// result, proof layout and error messages as the grand-sum prover; evalsSelF may be omitted (all ones).
const { prove } = require("../prover_common");
const backend = require("../backend");

module.exports = async function lookup_kzg_grandsum_prover(pTauFilename, evalsFs, evalsTs, evalsSelF = null, evalsMulT = null) {
    return prove(backend.LOOKUP, pTauFilename, evalsFs, evalsTs, evalsSelF, evalsMulT);
};
