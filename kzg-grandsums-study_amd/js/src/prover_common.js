// Shared body of the drop-in provers (grand-sum, grand-product, lookup): the reference's input checks (same messages,
// src/grandsum/mset_eq_kzg_prover.js:22-81), the HIP prover call, and the proof object with the
// reference's key names and insertion order.
const backend = require("./backend");
const logger = require("./logger");
const { Evaluations } = require("./polynomial/evaluations");
const { getCurveFromName } = require("./curve");

const TITLE = ["GRAND-SUM", "GRAND-PRODUCT", "GRAND-SUM (LOOKUP)"];

async function prove(kind, pTauFilename, evalsFs, evalsTs, evalsSelF, evalsSelT) {
    logger.info(`> MULTISET EQUALITY KZG ${TITLE[kind]} PROVER STARTED`);
    // the ptau header is read first, as the reference does (prover.js:15-16)
    const nBitsPTau = backend.ptauPower(pTauFilename);
    const curve = await getCurveFromName("bn128");
    if (!Array.isArray(evalsFs)) evalsFs = [evalsFs];
    if (!Array.isArray(evalsTs)) evalsTs = [evalsTs];
    if (evalsFs.length !== evalsTs.length) throw new Error(`The lengths of the two vector multisets must be the same.`);
    const nPols = evalsFs.length;
    if (nPols === 0) throw new Error(`The number of multisets must be greater than 0.`);
    for (let i = 0; i < nPols; i++) {
        if (evalsFs[i].length() !== evalsTs[i].length()) {
            throw new Error(`The ${i}-th multiset buffers must have the same length.`);
        } else if (evalsFs[i].length() !== evalsFs[0].length()) {
            throw new Error("The multiset buffers must all have the same length.");
        }
    }
    // absent selectors are all-ones vectors in the reference (prover.js:53-68): unselected, so they
    // need not be materialised; given ones are checked with the same rules and messages
    const noSelF = evalsSelF === null || evalsSelF === undefined;
    const noSelT = evalsSelT === null || evalsSelT === undefined;
    const isLookup = kind === backend.LOOKUP;
    if (isLookup && noSelT) throw new Error("A lookup needs the multiplicities of the table.");
    const lenSelF = noSelF ? evalsFs[0].length() : evalsSelF.length();
    const lenSelT = noSelT ? evalsTs[0].length() : evalsSelT.length();
    if (lenSelF !== lenSelT) {
        throw new Error("The selection buffers must have the same length.");
    } else if (lenSelF !== evalsFs[0].length()) {
        throw new Error("The selection buffers must have the same length as the multiset buffers.");
    }
    // a lookup keeps its selectors even when all one (its proof always carries selF / selT)
    let isSelected = true;
    if (!isLookup && (noSelF || evalsSelF.isAllOnes()) && (noSelT || evalsSelT.isAllOnes())) {
        isSelected = false;
    } else if (!noSelF && !noSelT && evalsSelF.isAllZeros() && evalsSelT.isAllZeros()) {
        logger.warn("The selection buffers are all zeros. The argument is trivially satisfied.");  // prover.js:66-68
    }
    if (isSelected) {
        if (noSelF) evalsSelF = Evaluations.getOneEvals(lenSelF, curve);
        if (noSelT) evalsSelT = Evaluations.getOneEvals(lenSelT, curve);
    }
    const nBits = Math.ceil(Math.log2(evalsFs[0].length()));
    if (evalsFs[0].length() !== 2 ** nBits) throw new Error("Polynomial length must be a power of two.");
    if (nBitsPTau < nBits) throw new Error("The Powers of Tau file is not sufficiently large to commit the polynomials.");

    const logInfo = logger.enabled("INFO");
    if (logInfo) {  // prover.js:87-93
        logger.info("-------------------------------------");
        logger.info(`  MULTISET EQUALITY KZG ${TITLE[kind]} PROVER SETTINGS`);
        logger.info(`  Curve:       ${curve.name}`);
        logger.info(`  Domain size: ${2 ** nBits}`);
        logger.info(`  Number of polynomials: ${nPols}`);
        logger.info(`  Selectors: ${isSelected ? "Yes" : "No"}`);
        logger.info("-------------------------------------");
    }

    const res = await backend.prove(kind, pTauFilename, nBits,
        evalsFs.map(e => e.eval), evalsTs.map(e => e.eval),
        isSelected ? evalsSelF.eval : null, isSelected ? evalsSelT.eval : null);
    // prover.js:147-148: the caller's objects now hold Montgomery form
    for (let i = 0; i < nPols; i++) {
        evalsFs[i].eval = res.montF[i];
        evalsTs[i].eval = res.montT[i];
    }
    const isVector = nPols > 1;
    const gs = kind !== backend.GRANDPRODUCT;
    const proof = { evaluations: {}, commitments: {} };
    let c = 0;
    for (let i = 0; i < nPols; i++) {
        proof.commitments[isVector ? `F${i}` : "F"] = res.commitments[c++];
        proof.commitments[isVector ? `T${i}` : "T"] = res.commitments[c++];
    }
    if (isSelected) {
        proof.commitments["selF"] = res.commitments[c++];
        proof.commitments["selT"] = res.commitments[c++];
    }
    proof.commitments[gs ? "S" : "Z"] = res.commitments[c++];
    proof.commitments["Q"] = res.commitments[c++];
    proof.commitments["Wxi"] = res.commitments[c++];
    proof.commitments["Wxiw"] = res.commitments[c++];
    let e = 0;
    for (let i = 0; i < nPols; i++) {
        proof.evaluations[isVector ? `f${i}xi` : "fxi"] = res.evaluations[e++];
        if (gs) proof.evaluations[isVector ? `t${i}xi` : "txi"] = res.evaluations[e++];
    }
    if (isSelected) {
        proof.evaluations["selFxi"] = res.evaluations[e++];
        proof.evaluations["selTxi"] = res.evaluations[e++];
    }
    proof.evaluations[gs ? "sxiw" : "zxiw"] = res.evaluations[e++];
    // the proof is computed inside libkgs in one call, so the round log is written after it, in the
    // reference's order, with the challenges replayed from the proof
    if (logInfo) logRounds(kind, curve, proof, nBits, nPols, isSelected);
    return proof;
}

// src/Keccak256Transcript.js:7-53: commitments enter as G1.toRprUncompressed (64 B), scalars as
// Fr.toRprBE (32 B); a challenge is keccak256 of everything added so far, big-endian, mod r
class Transcript {
    constructor(curve) {
        this.curve = curve;
        this.parts = [];
    }
    addPolCommitment(p) {
        const b = new Uint8Array(64);
        this.curve.G1.toRprUncompressed(b, 0, p);
        this.parts.push(b);
    }
    addFieldElement(a) {
        const b = new Uint8Array(32);
        this.curve.Fr.toRprBE(b, 0, a);
        this.parts.push(b);
    }
    getChallenge() {
        const h = backend.load().keccak256(Buffer.concat(this.parts.map(b => Buffer.from(b))));
        let x = 0n;
        for (const byte of h) x = (x << 8n) | BigInt(byte);
        return this.curve.Fr.e(x);
    }
}

// The reference's round log (prover.js:111-140 with the lines of each round: :164-177, :198-230,
// :238-285, :293-317, :338-344, :411-412; grand-product prover.js the same with Z and without t(z))
function logRounds(kind, curve, proof, nBits, nPols, isSelected) {
    const Fr = curve.Fr, G1 = curve.G1;
    const gs = kind !== backend.GRANDPRODUCT;
    const isVector = nPols > 1;
    const C = proof.commitments, E = proof.evaluations;
    const tr = new Transcript(curve);
    let round = 1;
    // the reference's message keeps "${round}" literally (a plain-quoted string, prover.js:111)
    let msg = "> ROUND ${round}. Generate the witness polynomials";
    msg += isVector ? ` fᵢ,tᵢ ∈ 𝔽[X], for i ∈ [${nPols}]` : ` f,t ∈ 𝔽[X]`;
    if (isSelected) msg += ", and the selector polynomials fsel,tsel ∈ 𝔽[X]";
    logger.info(msg);
    for (let i = 0; i < nPols; i++) {
        const nF = isVector ? `F${i}` : "F", nT = isVector ? `T${i}` : "T";
        logger.info(`··· [${isVector ? `f${i + 1}(x)` : "f(x)"}]₁ =`, G1.toString(C[nF]));
        logger.info(`··· [${isVector ? `t${i + 1}(x)` : "t(x)"}]₁ =`, G1.toString(C[nT]));
        tr.addPolCommitment(C[nF]);
        tr.addPolCommitment(C[nT]);
    }
    if (isSelected) {
        logger.info(`··· [fsel(x)]₁ =`, G1.toString(C["selF"]));
        logger.info(`··· [tsel(x)]₁ =`, G1.toString(C["selT"]));
        tr.addPolCommitment(C["selF"]);
        tr.addPolCommitment(C["selT"]);
    }
    ++round;
    const SZ = gs ? "S" : "Z";
    logger.info(`> ROUND ${round}. Compute the grand-${gs ? "sum" : "product"} polynomial ${SZ} ∈ 𝔽[X]`);
    let beta = null;
    if (isVector) {
        beta = tr.getChallenge();
        logger.info("···      𝛃  =", Fr.toString(beta));
        tr.addFieldElement(beta);
    }
    const gamma = tr.getChallenge();
    logger.info("···      𝜸  =", Fr.toString(gamma));
    logger.info(`··· [${SZ}(x)]₁ =`, G1.toString(C[SZ]));
    ++round;
    logger.info(`> ROUND ${round}. Compute the quotient polynomial Q ∈ 𝔽[X]`);
    tr.addFieldElement(gamma);
    tr.addPolCommitment(C[SZ]);
    const alpha = tr.getChallenge();
    logger.info("···      𝜶  =", Fr.toString(alpha));
    logger.info(`··· [Q(x)]₁ =`, G1.toString(C["Q"]));
    ++round;
    logger.info(`> ROUND ${round}. Compute the evaluations of the polynomials`);
    tr.addFieldElement(alpha);
    tr.addPolCommitment(C["Q"]);
    const xi = tr.getChallenge();
    logger.info("···      𝔷  =", Fr.toString(xi));
    for (let i = 0; i < nPols; i++) {
        logger.info(`···   ${isVector ? `f${i + 1}(𝔷)` : "f(𝔷)"}  =`, Fr.toString(E[isVector ? `f${i}xi` : "fxi"]));
        if (gs) logger.info(`···   ${isVector ? `t${i + 1}(𝔷)` : "t(𝔷)"}  =`, Fr.toString(E[isVector ? `t${i}xi` : "txi"]));
    }
    if (isSelected) {
        logger.info(`···   fsel(𝔷)  =`, Fr.toString(E["selFxi"]));
        logger.info(`···   tsel(𝔷)  =`, Fr.toString(E["selTxi"]));
    }
    logger.info(`··· ${SZ}(𝔷·𝛚)  =`, Fr.toString(E[gs ? "sxiw" : "zxiw"]));
    ++round;
    logger.info(`> ROUND ${round}. Compute the opening proof polynomials W𝔷, W𝔷𝛚 ∈ 𝔽[X]`);
    tr.addFieldElement(xi);
    for (let i = 0; i < nPols; i++) {
        tr.addFieldElement(E[isVector ? `f${i}xi` : "fxi"]);
        if (gs) tr.addFieldElement(E[isVector ? `t${i}xi` : "txi"]);
    }
    if (isSelected) {
        tr.addFieldElement(E["selFxi"]);
        tr.addFieldElement(E["selTxi"]);
    }
    tr.addFieldElement(E[gs ? "sxiw" : "zxiw"]);
    const v = tr.getChallenge();
    logger.info("···      v  = ", Fr.toString(v));
    // polynomial_utils.js:1-19
    let xn = xi;
    for (let i = 0; i < nBits; i++) xn = Fr.square(xn);
    const ZHxi = Fr.sub(xn, Fr.one);
    const L1xi = Fr.div(ZHxi, Fr.mul(Fr.e(2 ** nBits), Fr.sub(xi, Fr.one)));
    logger.info("···  ZH(𝔷)  =", Fr.toString(ZHxi));
    logger.info("···  L₁(𝔷)  =", Fr.toString(L1xi));
    logger.info("··· [W𝔷(x)]₁   =", G1.toString(C["Wxi"]));
    logger.info("··· [W𝔷·𝛚(x)]₁ =", G1.toString(C["Wxiw"]));
    logger.info("");
    logger.info(`> MULTISET EQUALITY KZG ${TITLE[kind]} PROVER FINISHED`);
    return { beta, gamma, alpha, xi, v };
}

module.exports = { prove, Transcript, logRounds };
