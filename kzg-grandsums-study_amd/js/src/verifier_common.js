// Shared body of the drop-in verifiers (src/grandsum/mset_eq_kzg_verifier.js:9,
// src/grandproduct/mset_eq_kzg_verifier.js:9, and the lookup one): the proof's shape is read from its keys exactly as
// the reference does (nPols from /^F\d/, selectors from /^selF/), the values are laid out in the
// C-ABI order and checked by libkgs's native verifier (transcript replay + optimal-ate pairing).
//
// Log lines: the reference's, step by step (grandsum verifier.js:10-75,99,122,143,167-190 and the
// validation errors :192-204; grandproduct verifier.js the same with its own r0 / [D]1 lines and its
// "GRAND-SUM VERIFIER SETTINGS" header, kept verbatim). The challenges, ZH(xi), L1(xi), r0, [D]1,
// [F]1 and [E]1 are recomputed on the host with the curve shim, the reference's way, only when INFO
// lines reach an output; the accept / reject decision is the native verifier's.
const backend = require("./backend");
const logger = require("./logger");
const { getCurveFromName } = require("./curve");
const { Transcript } = require("./prover_common");

const TITLE = ["GRAND-SUM", "GRAND-PRODUCT", "GRAND-SUM (LOOKUP)"];

async function verify(kind, pTauFilename, proof, nBits) {
    logger.info(`> MULTISET EQUALITY KZG ${TITLE[kind]} VERIFIER STARTED`);
    const keys = Object.keys(proof.commitments);
    const nFi = keys.filter(k => k.match(/^F\d/)).length;
    const nPols = nFi > 0 ? nFi : 1;
    const isVector = nPols > 1;
    const isSelected = keys.filter(k => k.match(/^selF/)).length === 1;
    const gs = kind !== backend.GRANDPRODUCT;
    const SZ = gs ? "S" : "Z";
    const curve = await getCurveFromName("bn128");
    const Fr = curve.Fr, G1 = curve.G1;

    logger.info("---------------------------------------");
    // the grand-product reference prints the grand-sum header here (grandproduct verifier.js:31)
    logger.info("  MULTISET EQUALITY KZG GRAND-SUM VERIFIER SETTINGS");
    logger.info(`  Curve:        ${curve.name}`);
    logger.info(`  Domain size:  ${2 ** nBits}`);
    logger.info(`  #polynomials: ${nPols}`);
    logger.info(`  Selectors:    ${isSelected ? "Yes" : "No"}`);
    logger.info("---------------------------------------");
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
    cNames.push(SZ, "Q", "Wxi", "Wxiw");
    eNames.push(gs ? "sxiw" : "zxiw");
    // a missing member is a malformed proof object: the reference's G1.isValid / Scalar.fromRprLE
    // on `undefined` throws, so this does too (a present but wrong-sized value just fails to verify)
    for (const n of cNames)
        if (proof.commitments[n] === undefined || proof.commitments[n] === null)
            throw new TypeError(`proof.commitments.${n} is missing`);
    for (const n of eNames)
        if (proof.evaluations[n] === undefined || proof.evaluations[n] === null)
            throw new TypeError(`proof.evaluations.${n} is missing`);

    let step = 1;
    let pols = "";
    if (isVector) for (let i = 0; i < nPols; i++) pols += `[f${i + 1}(x)]₁,[t${i + 1}(x)]₁,`;
    if (isSelected) pols += "[fsel(x)]₁,[tsel(x)]₁,";
    logger.info(`> STEP ${step}. Validate ${pols}[${SZ}(x)]₁,[Q(x)]₁,[W𝔷(x)]₁,[W𝔷·𝛚(x)]₁ ∈ 𝔾₁`);
    const C = proof.commitments, E = proof.evaluations;
    const g1Ok = (name, v) => {
        const ok = v instanceof Uint8Array && (v.length === 64 || v.length === 96) && G1.isValid(v);
        if (!ok) logger.error(`··· ERROR: ${name} is not a valid G1 element`, v instanceof Uint8Array && v.length >= 64 ? G1.toString(v) : String(v));
        return ok;
    };
    const frOk = (name, v) => {
        let ok = v instanceof Uint8Array && v.length === 32;
        if (ok) {
            let x = 0n;
            for (let i = 31; i >= 0; i--) x = (x << 8n) | BigInt(v[i]);
            ok = x < BigInt(Fr.p);
        }
        if (!ok) logger.error(`··· ERROR: ${name} is not a valid field element`, v instanceof Uint8Array && v.length === 32 ? Fr.toString(v) : String(v));
        return ok;
    };
    for (let i = 0; i < nPols; i++) {
        if (!g1Ok(`[${isVector ? `f${i + 1}(x)` : "f(x)"}]₁`, C[isVector ? `F${i}` : "F"])) return false;
        if (!g1Ok(`[${isVector ? `t${i + 1}(x)` : "t(x)"}]₁`, C[isVector ? `T${i}` : "T"])) return false;
    }
    if (isSelected && (!g1Ok("[fsel(x)]₁", C["selF"]) || !g1Ok("[tsel(x)]₁", C["selT"]))) return false;
    if (!(g1Ok(`[${SZ}(x)]₁`, C[SZ]) && g1Ok("[Q(x)]₁", C["Q"]) && g1Ok("[W𝔷(x)]₁", C["Wxi"]) &&
          g1Ok("[W𝔷·𝛚(x)]₁", C["Wxiw"]))) return false;
    ++step;

    let evals = "";
    if (isVector) for (let i = 0; i < nPols; i++) evals += gs ? `f${i + 1}(𝔷),t${i + 1}(𝔷),` : `f${i + 1}(𝔷),`;
    if (isSelected) evals += "fsel(𝔷),tsel(𝔷),";
    logger.info(`> STEP ${step}. Validate ${evals},${SZ}(𝔷·𝛚) ∈ 𝔽`);
    for (let i = 0; i < nPols; i++) {
        if (!frOk(isVector ? `f${i + 1}(𝔷)` : "f(𝔷)", E[isVector ? `f${i}xi` : "fxi"])) return false;
        if (gs && !frOk(isVector ? `t${i + 1}(𝔷)` : "t(𝔷)", E[isVector ? `t${i}xi` : "txi"])) return false;
    }
    if (!frOk(`${SZ}(𝔷·𝛚)`, E[gs ? "sxiw" : "zxiw"])) return false;
    ++step;

    if (logger.enabled("INFO")) logSteps(kind, curve, proof, nBits, nPols, isSelected, step);

    const com = new Uint8Array(64 * cNames.length);
    cNames.forEach((n, i) => com.set(C[n].length === 64 ? C[n] : G1.toAffine(C[n]), 64 * i));
    const ev = new Uint8Array(32 * eNames.length);
    eNames.forEach((n, i) => ev.set(E[n], 32 * i));
    const isValid = backend.load().verifyPtau(kind, require("path").resolve(pTauFilename), nBits, nPols, isSelected, com, ev);
    if (isValid) logger.info("> VERIFICATION OK");
    else logger.error("> VERIFICATION FAILED");
    logger.info(`> MULTISET EQUALITY KZG ${TITLE[kind]} VERIFIER FINISHED`);
    return isValid;
}

// STEP 3 .. 9 of the reference's verifier, their values computed its way (host BigInt arithmetic)
function logSteps(kind, curve, proof, nBits, nPols, isSelected, step) {
    const Fr = curve.Fr, G1 = curve.G1;
    const gs = kind !== backend.GRANDPRODUCT;
    const lookup = kind === backend.LOOKUP;
    const isVector = nPols > 1;
    const C = proof.commitments, E = proof.evaluations;
    const SZ = gs ? "S" : "Z";
    const szxiw = E[gs ? "sxiw" : "zxiw"];
    const fName = (i) => (isVector ? `f${i}xi` : "fxi"), tName = (i) => (isVector ? `t${i}xi` : "txi");
    const FName = (i) => (isVector ? `F${i}` : "F"), TName = (i) => (isVector ? `T${i}` : "T");

    logger.info(`> STEP ${step}. Compute ${isVector ? "𝛽," : ""}𝜸,𝜶,𝔷,v,u`);
    const ch = {};
    const tr = new Transcript(curve);
    for (let i = 0; i < nPols; i++) {
        tr.addPolCommitment(C[FName(i)]);
        tr.addPolCommitment(C[TName(i)]);
    }
    if (isSelected) {
        tr.addPolCommitment(C["selF"]);
        tr.addPolCommitment(C["selT"]);
    }
    if (isVector) {
        ch.beta = tr.getChallenge();
        logger.info("··· 𝛃 =", Fr.toString(ch.beta));
        tr.addFieldElement(ch.beta);
    }
    ch.gamma = tr.getChallenge();
    logger.info("··· 𝜸 =", Fr.toString(ch.gamma));
    tr.addFieldElement(ch.gamma);
    tr.addPolCommitment(C[SZ]);
    ch.alpha = tr.getChallenge();
    logger.info("··· 𝜶 =", Fr.toString(ch.alpha));
    tr.addFieldElement(ch.alpha);
    tr.addPolCommitment(C["Q"]);
    ch.xi = tr.getChallenge();
    logger.info("··· 𝔷 =", Fr.toString(ch.xi));
    tr.addFieldElement(ch.xi);
    for (let i = 0; i < nPols; i++) {
        tr.addFieldElement(E[fName(i)]);
        if (gs) tr.addFieldElement(E[tName(i)]);
    }
    if (isSelected) {
        tr.addFieldElement(E["selFxi"]);
        tr.addFieldElement(E["selTxi"]);
    }
    tr.addFieldElement(szxiw);
    ch.v = tr.getChallenge();
    logger.info("··· v =", Fr.toString(ch.v));
    tr.addFieldElement(ch.v);
    tr.addPolCommitment(C["Wxi"]);
    tr.addPolCommitment(C["Wxiw"]);
    ch.u = tr.getChallenge();
    logger.info("··· u =", Fr.toString(ch.u));
    // a single-vector proof has no beta; it only ever multiplies a zero accumulator
    const beta = ch.beta || Fr.zero;
    ++step;

    logger.info(`> STEP ${step}. Compute ZH(𝔷) and L₁(𝔷)`);
    let xn = ch.xi;
    for (let i = 0; i < nBits; i++) xn = Fr.square(xn);
    const ZHxi = Fr.sub(xn, Fr.one);
    const L1xi = Fr.div(ZHxi, Fr.mul(Fr.e(2 ** nBits), Fr.sub(ch.xi, Fr.one)));
    logger.info("··· ZH(𝔷) =", Fr.toString(ZHxi));
    logger.info("··· L₁(𝔷) =", Fr.toString(L1xi));
    ++step;

    logger.info(gs ? `> STEP ${step}. Compute r₀ = `
                   : `> STEP ${step}. Compute r₀ = -L₁(𝔷) + 𝜶[Z(𝔷·𝛚)(tsel(𝔷)(𝜸 - 1) + 1)] + 𝜶²[fsel(𝔷)(1 - fsel(𝔷))] + 𝜶³[tsel(𝔷)(1 - tsel(𝔷))]`);
    let r0 = Fr.zero;
    if (isSelected) {
        // the lookup's selT holds multiplicities: no binary term for it (DESIGN.md §0 row N4)
        const selTBin = lookup ? Fr.zero : Fr.sub(E["selTxi"], Fr.square(E["selTxi"]));
        r0 = Fr.mul(Fr.add(r0, selTBin), ch.alpha);
        const selFBin = Fr.sub(E["selFxi"], Fr.square(E["selFxi"]));
        r0 = Fr.mul(Fr.add(r0, selFBin), ch.alpha);
    }
    let D1;
    if (gs) {
        let fxi = Fr.zero, txi = Fr.zero;
        for (let i = nPols - 1; i >= 0; i--) {
            fxi = Fr.add(Fr.mul(fxi, beta), E[fName(i)]);
            txi = Fr.add(Fr.mul(txi, beta), E[tName(i)]);
        }
        const fxigamma = Fr.add(fxi, ch.gamma), txigamma = Fr.add(txi, ch.gamma);
        let r01 = Fr.mul(szxiw, Fr.mul(fxigamma, txigamma));
        if (isSelected) {
            r01 = Fr.add(r01, Fr.mul(E["selTxi"], fxigamma));
            r01 = Fr.sub(r01, Fr.mul(E["selFxi"], txigamma));
        } else {
            r01 = Fr.sub(Fr.add(r01, fxi), txi);
        }
        r0 = Fr.mul(Fr.add(r0, r01), ch.alpha);
        logger.info("··· r₀    =", Fr.toString(r0));
        ++step;
        logger.info(`> STEP ${step}. Compute [D]₁ = `);
        const D1_12 = Fr.mul(Fr.mul(ch.alpha, fxigamma), txigamma);
        const D1_1 = G1.timesFr(C["S"], Fr.add(Fr.sub(L1xi, D1_12), ch.u));
        D1 = G1.sub(D1_1, G1.timesFr(C["Q"], ZHxi));
    } else {
        let r01 = szxiw;
        if (isSelected) r01 = Fr.mul(r01, Fr.add(Fr.mul(Fr.sub(ch.gamma, Fr.one), E["selTxi"]), Fr.one));
        else r01 = Fr.mul(r01, ch.gamma);
        r0 = Fr.sub(Fr.mul(Fr.add(r0, r01), ch.alpha), L1xi);
        logger.info("··· r₀    =", Fr.toString(r0));
        ++step;
        logger.info(`> STEP ${step}. Compute [D]₁ = `);
        let fxi = Fr.zero;
        for (let i = nPols - 1; i >= 0; i--) fxi = Fr.add(Fr.mul(fxi, beta), E[fName(i)]);
        let fxigamma = Fr.add(fxi, ch.gamma);
        if (isSelected) fxigamma = Fr.add(Fr.mul(Fr.sub(fxigamma, Fr.one), E["selFxi"]), Fr.one);
        const D1_1 = G1.timesFr(C["Z"], Fr.add(Fr.sub(L1xi, Fr.mul(ch.alpha, fxigamma)), ch.u));
        let D1_2 = G1.zero;
        for (let i = nPols - 1; i >= 0; i--) D1_2 = G1.add(G1.timesFr(D1_2, beta), C[TName(i)]);
        if (isSelected) D1_2 = G1.timesFr(D1_2, E["selTxi"]);
        D1_2 = G1.timesFr(G1.timesFr(D1_2, szxiw), ch.alpha);
        D1 = G1.sub(G1.add(D1_1, D1_2), G1.timesFr(C["Q"], ZHxi));
    }
    logger.info("··· [D]₁  =", G1.toString(G1.toAffine(D1)));
    ++step;

    logger.info(`> STEP ${step}. Compute [F]₁ = `);
    let F1 = G1.zero;
    if (isSelected) {
        F1 = G1.add(F1, C["selT"]);
        F1 = G1.add(G1.timesFr(F1, ch.v), C["selF"]);
    }
    if (gs) for (let i = nPols - 1; i >= 0; i--) F1 = G1.add(G1.timesFr(F1, ch.v), C[TName(i)]);
    for (let i = nPols - 1; i >= 0; i--) F1 = G1.add(G1.timesFr(F1, ch.v), C[FName(i)]);
    F1 = G1.add(G1.timesFr(F1, ch.v), D1);
    logger.info("··· [F]₁  =", G1.toString(G1.toAffine(F1)));
    ++step;

    logger.info(`> STEP ${step}. Compute [E]₁ = `);
    let E1 = Fr.zero;
    if (isSelected) {
        E1 = Fr.add(E1, E["selTxi"]);
        E1 = Fr.add(Fr.mul(E1, ch.v), E["selFxi"]);
    }
    if (gs) for (let i = nPols - 1; i >= 0; i--) E1 = Fr.add(Fr.mul(E1, ch.v), E[tName(i)]);
    for (let i = nPols - 1; i >= 0; i--) E1 = Fr.add(Fr.mul(E1, ch.v), E[fName(i)]);
    E1 = Fr.sub(Fr.add(Fr.mul(E1, ch.v), Fr.mul(ch.u, szxiw)), r0);
    logger.info("··· [E]₁  =", G1.toString(G1.toAffine(G1.timesFr(G1.one, E1))));
    ++step;

    logger.info(`> STEP ${step}. Check pairing equation e(-[W𝔷(x)]₁ - u·[W𝔷·𝛚(x)]₁, [x]₂)·e(𝔷·[W𝔷(x)]₁ + u𝔷ω·[W𝔷·𝛚(x)]₁ + [F]₁ - [E]₁, [1]₂) = 1`);
}

module.exports = { verify };
