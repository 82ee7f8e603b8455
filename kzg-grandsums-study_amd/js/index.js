// JavaScript host of the MI355X prover: the reference's module surface.
module.exports = {
    getCurveFromName: require("./src/curve").getCurveFromName,
    BigBuffer: require("./src/bigbuffer").BigBuffer,
    Scalar: require("./src/scalar").Scalar,
    Evaluations: require("./src/polynomial/evaluations").Evaluations,
    mset_eq_kzg_grandsum_prover: require("./src/grandsum/mset_eq_kzg_prover"),
    mset_eq_kzg_grandproduct_prover: require("./src/grandproduct/mset_eq_kzg_prover"),
    mset_eq_kzg_grandsum_verifier: require("./src/grandsum/mset_eq_kzg_verifier"),
    mset_eq_kzg_grandproduct_verifier: require("./src/grandproduct/mset_eq_kzg_verifier"),
    lookup_kzg_grandsum_prover: require("./src/lookup/lookup_kzg_prover"),
    lookup_kzg_grandsum_verifier: require("./src/lookup/lookup_kzg_verifier"),
    // the provers' log channel (the reference's logger.js lines): setLogger(logplease instance), setLogLevel
    logger: require("./src/logger"),
};
