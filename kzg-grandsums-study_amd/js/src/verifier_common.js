// Shared body of the drop-in verifiers (src/grandsum/mset_eq_kzg_verifier.js:9,
// src/grandproduct/mset_eq_kzg_verifier.js:9, and the lookup one): the proof's shape is read from its keys exactly as
// the reference does (nPols from /^F\d/, selectors from /^selF/), the values are laid out in the
// C-ABI order and checked by libkgs's native verifier (transcript replay + optimal-ate pairing).
const backend = require("./backend");

async function verify(kind, pTauFilename, proof, nBits) {
    const keys = Object.keys(proof.commitments);
    const nFi = keys.filter(k => k.match(/^F\d/)).length;
    const nPols = nFi > 0 ? nFi : 1;
    const isVector = nPols > 1;
    const isSelected = keys.filter(k => k.match(/^selF/)).length === 1;
    const gs = kind !== backend.GRANDPRODUCT;
    if (kind === backend.LOOKUP && !isSelected) return false;
    const cNames = [], eNames = [];
    for (let i = 0; i < nPols; i++) {
        cNames.push(isVector ? `F${i}` : "F", isVector ? `T${i}` : "T");
        eNames.push(isVector ? `f${i}xi` : "fxi");
        if (gs) eNames.push(isVector ? `t${i}xi` : "txi");
    }
    if (isSelected) {
        cNames.push("selF", "selT");
        eNames.push("selFxi", "selTxi");
    }
    cNames.push(gs ? "S" : "Z", "Q", "Wxi", "Wxiw");
    eNames.push(gs ? "sxiw" : "zxiw");
    for (const n of cNames) if (!(proof.commitments[n] instanceof Uint8Array) || proof.commitments[n].length !== 64) return false;
    for (const n of eNames) if (!(proof.evaluations[n] instanceof Uint8Array) || proof.evaluations[n].length !== 32) return false;
    const com = new Uint8Array(64 * cNames.length);
    cNames.forEach((n, i) => com.set(proof.commitments[n], 64 * i));
    const ev = new Uint8Array(32 * eNames.length);
    eNames.forEach((n, i) => ev.set(proof.evaluations[n], 32 * i));
    return backend.load().verifyPtau(kind, require("path").resolve(pTauFilename), nBits, nPols, isSelected, com, ev);
}

module.exports = { verify };
