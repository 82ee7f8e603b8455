// Shared body of the drop-in provers (grand-sum, grand-product, lookup): the reference's input checks (same messages,
// src/grandsum/mset_eq_kzg_prover.js:22-81), the HIP prover call, and the proof object with the
// reference's key names and insertion order.
const backend = require("./backend");
const { Evaluations } = require("./polynomial/evaluations");
const { getCurveFromName } = require("./curve");

async function prove(kind, pTauFilename, evalsFs, evalsTs, evalsSelF, evalsSelT) {
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
    if (!isLookup && (noSelF || evalsSelF.isAllOnes()) && (noSelT || evalsSelT.isAllOnes())) isSelected = false;
    if (isSelected) {
        if (noSelF) evalsSelF = Evaluations.getOneEvals(lenSelF, curve);
        if (noSelT) evalsSelT = Evaluations.getOneEvals(lenSelT, curve);
    }
    const nBits = Math.ceil(Math.log2(evalsFs[0].length()));
    if (evalsFs[0].length() !== 2 ** nBits) throw new Error("Polynomial length must be a power of two.");
    if (nBitsPTau < nBits) throw new Error("The Powers of Tau file is not sufficiently large to commit the polynomials.");

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
    return proof;
}

module.exports = { prove };
