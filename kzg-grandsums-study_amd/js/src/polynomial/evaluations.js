// Evaluation-form vector: the prover's input container. Same surface as the reference's
// src/polynomial/evaluations.js:5-136 (fromArray, fromEvals, getOneEvals, getZeroEvals,
// getRandomEvals, getRandomBinEvals, getEvaluation, getEvaluationSequence, setEvaluation, length,
// isEqual, isAllZeros, isAllOnes). `fromPolynomial` (the fft helper) is not needed by callers: the
// prover's NTTs run on the GPU.
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
    static fromEvals(evals) { return new Evaluations(evals.eval.slice(), evals.curve); }
    static getOneEvals(length, curve) {
        const buffer = new Uint8Array(length * curve.Fr.n8);
        for (let i = 0; i < length; i++) buffer.set(curve.Fr.one, i * curve.Fr.n8);
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
        return length;
    }
    isEqual(other) {
        if (this.length() !== other.length()) return false;
        return Buffer.compare(Buffer.from(this.eval), Buffer.from(other.eval)) === 0;
    }
    isAllZeros() { return this.isEqual(new Evaluations(new Uint8Array(this.length() * this.Fr.n8), this.curve)); }
    isAllOnes() { return this.isEqual(Evaluations.getOneEvals(this.length(), this.curve)); }
}

module.exports = { Evaluations };
