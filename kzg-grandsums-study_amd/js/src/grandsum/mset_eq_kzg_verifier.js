// Drop-in for src/grandsum/mset_eq_kzg_verifier.js:9 — same export, arguments and Promise<boolean>.
const { verify } = require("../verifier_common");
const backend = require("../backend");

module.exports = async function mset_eq_kzg_grandsum_verifier(pTauFilename, proof, nBits) {
    return verify(backend.GRANDSUM, pTauFilename, proof, nBits);
};
