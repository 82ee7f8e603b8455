// Verifier of lookup_kzg_prover's proofs: the grand-sum verifier (src/grandsum/mset_eq_kzg_verifier.js:9)
// without the selT-binary term of r0 (:80-81), run natively by libkgs (kgs_verify_ptau, KGS_LOOKUP).
const { verify } = require("../verifier_common");
const backend = require("../backend");

module.exports = async function lookup_kzg_grandsum_verifier(pTauFilename, proof, nBits) {
    return verify(backend.LOOKUP, pTauFilename, proof, nBits);
};
