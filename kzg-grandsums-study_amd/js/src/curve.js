// Minimal BN254 ("bn128") curve shim: exactly the members the reference modules and their callers
// touch (SURVEY.md §8b): Fr {n8, p, zero, one, negone, two, w[], e, add, sub, mul, neg, square, inv,
// div, eq, isZero, random, toString, toRprBE, toRprLE}, G1.F.n8, name, terminate. Field elements are
// 32-byte little-endian Montgomery Uint8Arrays (ffjavascript's in-memory form). BigInt arithmetic:
// this is host plumbing only; the hot path runs on the GPU through the addon.
const crypto = require("crypto");

const R = 21888242871839275222246405745257275088548364400416034343698204186575808495617n;
const Q = 21888242871839275222246405745257275088696311157297823662689037894645226208583n;
const MONT = 1n << 256n;

function modpow(b, e, m) {
    let r = 1n;
    b %= m;
    while (e > 0n) {
        if (e & 1n) r = (r * b) % m;
        b = (b * b) % m;
        e >>= 1n;
    }
    return r;
}

function toLE(x) {
    const out = new Uint8Array(32);
    for (let i = 0; i < 32; i++) { out[i] = Number(x & 0xffn); x >>= 8n; }
    return out;
}
function fromLE(b) {
    let x = 0n;
    for (let i = 31; i >= 0; i--) x = (x << 8n) | BigInt(b[i]);
    return x;
}

class Field {
    constructor(p) {
        this.p = p;
        this.n8 = 32;
        this.Rinv = modpow(MONT % p, p - 2n, p);
        this.zero = this.e(0n);
        this.one = this.e(1n);
        this.two = this.e(2n);
        this.negone = this.e(p - 1n);
    }
    // standard bigint -> Montgomery bytes
    e(a, base) {
        let v = typeof a === "bigint" ? a : BigInt(typeof a === "string" && base ? parseInt(a, base) : a);
        v %= this.p;
        if (v < 0n) v += this.p;
        return toLE((v * MONT) % this.p);
    }
    toObject(a) { return (fromLE(a) * this.Rinv) % this.p; }
    add(a, b) { return this.e(this.toObject(a) + this.toObject(b)); }
    sub(a, b) { return this.e(this.toObject(a) - this.toObject(b)); }
    mul(a, b) { return this.e(this.toObject(a) * this.toObject(b)); }
    square(a) { return this.mul(a, a); }
    neg(a) { return this.e(-this.toObject(a)); }
    inv(a) { return this.e(modpow(this.toObject(a), this.p - 2n, this.p)); }
    div(a, b) { return this.mul(a, this.inv(b)); }
    eq(a, b) { return Buffer.compare(Buffer.from(a), Buffer.from(b)) === 0; }
    isZero(a) { return this.toObject(a) === 0n; }
    random() { return this.e(fromLE(crypto.randomBytes(32)) % this.p); }
    toString(a, radix = 10) { return this.toObject(a).toString(radix); }
    toRprLE(buff, o, a) { buff.set(toLE(this.toObject(a)), o); }
    toRprBE(buff, o, a) { buff.set(toLE(this.toObject(a)).reverse(), o); }
}

function buildBn128() {
    const Fr = new Field(R);
    const F1 = new Field(Q);
    // Fr.w[k]: primitive 2^k-th roots, nqr = 5, s = 28
    Fr.s = 28;
    Fr.w = new Array(29);
    let w = modpow(5n, (R - 1n) >> 28n, R);
    for (let k = 28; k >= 0; k--) { Fr.w[k] = Fr.e(w); w = (w * w) % R; }
    return {
        name: "bn128",
        Fr,
        F1,
        G1: { F: { n8: 32 } },
        G2: { F: { n8: 64 } },
        terminate: async () => {},
    };
}

let cached = null;
async function getCurveFromName(name) {
    const n = String(name).toUpperCase().replace(/[^A-Z0-9]/g, "");
    if (!["BN128", "BN254", "ALTBN128"].includes(n)) throw new Error(`Curve not supported: ${name}`);
    if (!cached) cached = buildBn128();
    return cached;
}

module.exports = { getCurveFromName, R, Q };
