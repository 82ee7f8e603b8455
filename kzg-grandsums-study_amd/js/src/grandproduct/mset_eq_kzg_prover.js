// Drop-in for src/grandproduct/mset_eq_kzg_prover.js:12 (see ../grandsum/mset_eq_kzg_prover.js).
const { prove } = require("../prover_common");
const backend = require("../backend");

module.exports = async function mset_eq_kzg_grandproduct_prover(pTauFilename, evalsFs, evalsTs, evalsSelF = null, evalsSelT = null) {
    return prove(backend.GRANDPRODUCT, pTauFilename, evalsFs, evalsTs, evalsSelF, evalsSelT);
};
