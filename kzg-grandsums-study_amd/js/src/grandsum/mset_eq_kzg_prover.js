// Drop-in for src/grandsum/mset_eq_kzg_prover.js:12 — same export, arguments, Promise result and
// error messages; the prover chain runs on the MI355X through libkgs (include/kgs.h).
const { prove } = require("../prover_common");
const backend = require("../backend");

module.exports = async function mset_eq_kzg_grandsum_prover(pTauFilename, evalsFs, evalsTs, evalsSelF = null, evalsSelT = null) {
    return prove(backend.GRANDSUM, pTauFilename, evalsFs, evalsTs, evalsSelF, evalsSelT);
};
