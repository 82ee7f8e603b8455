// Evaluation-form vector: the prover's input container. Same surface as the reference's
// src/polynomial/evaluations.js:5-136 (fromArray, fromEvals, getOneEvals, getZeroEvals,
// getRandomEvals, getRandomBinEvals, getEvaluation, getEvaluationSequence, setEvaluation, length,
// isEqual, isAllZeros, isAllOnes, print), and fromPolynomial through the curve shim's GPU Fr.fft.
// The prover itself does not use fromPolynomial: its NTTs run inside libkgs.
const { BigBuffer } = require("../bigbuffer");
const logger = require("../logger");

class Evaluations {
    constructor(evaluations, curve) {
        this.eval = evaluations;
        this.curve = curve;
        this.Fr = curve.Fr;
    }
    static fromArray(array, curve) {
        const buffer = new Uint8Array(array.length * curve.Fr.n8);
        for (let i = 0; i < array.length; i++) buffer.set(array[i], i * curve.Fr.n8);
        return new Evaluations(buffer, curve);
    }
    // evaluations.js:12-21: zero-pad the coefficients (by buffer length, not degree) to
    // 2^ceil(log2 len) * extension and take the forward DFT
    static async fromPolynomial(polynomial, extension, curve) {
        const power = Math.ceil(Math.log2(polynomial.length()));
        const length = (1 << power) * extension;
        const coefficientsN = new BigBuffer(length * curve.Fr.n8);
        coefficientsN.set(polynomial.coef, 0);
        return new Evaluations(await curve.Fr.fft(coefficientsN), curve);
    }
    static fromEvals(evals) { return new Evaluations(evals.eval.slice(), evals.curve); }
    static getOneEvals(length, curve) {
        const n8 = curve.Fr.n8, buffer = new Uint8Array(length * n8);
        if (length > 0) {
            buffer.set(curve.Fr.one, 0);
            for (let filled = n8; filled < buffer.length; filled *= 2)  // doubling copies (memcpy)
                buffer.copyWithin(filled, 0, Math.min(filled, buffer.length - filled));
        }
        return new Evaluations(buffer, curve);
    }
    static getZeroEvals(length, curve) { return new Evaluations(new Uint8Array(length * curve.Fr.n8), curve); }
    static getRandomEvals(length, curve) {
        const buffer = new Uint8Array(length * curve.Fr.n8);
        for (let i = 0; i < length; i++) buffer.set(curve.Fr.random(), i * curve.Fr.n8);
        return new Evaluations(buffer, curve);
    }
    static getRandomBinEvals(length, curve) {
        const buffer = new Uint8Array(length * curve.Fr.n8);
        for (let i = 0; i < length; i++) buffer.set(Math.random() < 0.5 ? curve.Fr.one : curve.Fr.zero, i * curve.Fr.n8);
        return new Evaluations(buffer, curve);
    }
    getEvaluation(index) {
        if ((index + 1) * this.Fr.n8 > this.eval.byteLength) throw new Error("Evaluations.getEvaluation() out of bounds");
        return this.eval.slice(index * this.Fr.n8, (index + 1) * this.Fr.n8);
    }
    getEvaluationSequence(start, end) {
        if (start > end) throw new Error("Evaluations.getEvaluationSequence() start index is greater than end index");
        else if (start === end) throw new Error("Use Evaluations.getEvaluation() instead");
        if (end > this.length() - 1) throw new Error("Evaluations.getEvaluationSequence() end index is out of bounds");
        return this.eval.slice(start * this.Fr.n8, end * this.Fr.n8);
    }
    setEvaluation(index, value) {
        if (index > this.length() - 1) throw new Error("Evaluation index is out of bounds");
        this.eval.set(value, index * this.Fr.n8);
    }
    length() {
        const length = this.eval.byteLength / this.Fr.n8;
        if (length !== Math.floor(length)) throw new Error("Polynomial evaluations buffer has incorrect size");
        if (length === 0) logger.warn("Polynomial has length zero");  // evaluations.js:104-106
        return length;
    }
    isEqual(other) {
        if (this.length() !== other.length()) return false;
        return Buffer.compare(view(this.eval), view(other.eval)) === 0;
    }
    // every element equals the first one: element 0 matches, and the vector equals itself shifted by
    // one element (one native compare, no second vector)
    isConstant(value) {
        const n8 = this.Fr.n8, b = view(this.eval);
        if (this.length() === 0) return true;  // (the reference's warning, through length())
        if (Buffer.compare(b.subarray(0, n8), view(value)) !== 0) return false;
        return Buffer.compare(b.subarray(n8), b.subarray(0, b.length - n8)) === 0;
    }
    isAllZeros() { return this.isConstant(this.Fr.zero); }
    isAllOnes() { return this.isConstant(this.Fr.one); }
    // evaluations.js:131-135: one stdout line per element, "<name>(𝛚^i) = <decimal value>"
    print(name = "f") {
        for (let i = 0; i < this.length(); i++)
            console.log(`${name}(𝛚^${i}) =`, this.Fr.toString(this.getEvaluation(i)));
    }
}

// Buffer over a Uint8Array's memory (no copy, unlike Buffer.from(typedArray))
function view(u8) { return Buffer.from(u8.buffer, u8.byteOffset, u8.byteLength); }

module.exports = { Evaluations };
