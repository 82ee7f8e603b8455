// BN254 ("bn128") curve shim with the members the reference modules and their callers touch
// (SURVEY.md §8b), in ffjavascript's in-memory formats:
//   Fr, F1 {n8, p, zero, one, negone, two, w[], e, add, sub, mul, neg, square, inv, div, eq, isZero,
//           random, toString, toRprBE, toRprLE, toObject, fromMontgomery, toMontgomery}
//   Fr     {fft, ifft, batchInverse, batchToMontgomery, batchFromMontgomery}: on the GPU through the
//           addon (kgs_ntt / kgs_fr_batch_inverse / kgs_fr_to_mont / kgs_fr_from_mont), Promises of
//           the input's buffer kind (Uint8Array, or BigBuffer for a BigBuffer)
//   G1 {F, zero, one, zeroAffine, oneAffine, add, sub, neg, double, eq, isZero, timesFr,
//       timesScalar, toAffine, toJacobian, isValid, toRprUncompressed, fromRprUncompressed,
//       toRprLEM, fromRprLEM, toObject, fromObject, toString, multiExpAffine}
//   G2 {F, one, oneAffine, toAffine, fromRprLEM, toRprLEM}, pairingEq, name, terminate.
// Field elements are 32-byte little-endian Montgomery Uint8Arrays; G1 points are 96 B Jacobian
// (x, y, z; z = 0 for the zero point) or 64 B affine (x, y; (0, 0) = zero), G2 points 192 B / 128 B
// over Fq2 (c0, c1). Group arithmetic here is BigInt host plumbing (the verifier's handful of point
// operations); G1.multiExpAffine runs on the GPU through the addon (kgs_msm over the given bases)
// and curve.pairingEq through the native optimal-ate pairing (kgs_pairing_eq). The hot path itself
// is libkgs's prover.
const crypto = require("crypto");
const { BigBuffer, contiguous } = require("./bigbuffer");

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
    fromMontgomery(a) { return toLE(this.toObject(a)); }
    toMontgomery(a) { return this.e(fromLE(a)); }
}

// ---------------------------------------------------------------- G1 (y^2 = x^3 + 3 over Fq)
// internal form: Jacobian BigInt triple [x, y, z] in standard form; z = 0n is the zero point
const G1_B = 3n;
const md = (a) => { const r = a % Q; return r < 0n ? r + Q : r; };
const qinv = (a) => modpow(md(a), Q - 2n, Q);

function jacDouble(P) {
    const [x, y, z] = P;
    if (z === 0n || y === 0n) return [0n, 1n, 0n];
    const a = md(x * x), b = md(y * y), c = md(b * b);
    const d = md(2n * (md((x + b) * (x + b)) - a - c));
    const e = md(3n * a), f = md(e * e);
    const x3 = md(f - 2n * d);
    const y3 = md(e * (d - x3) - 8n * c);
    const z3 = md(2n * y * z);
    return [x3, y3, z3];
}

function jacAdd(P, R) {
    if (P[2] === 0n) return R;
    if (R[2] === 0n) return P;
    const z1z1 = md(P[2] * P[2]), z2z2 = md(R[2] * R[2]);
    const u1 = md(P[0] * z2z2), u2 = md(R[0] * z1z1);
    const s1 = md(P[1] * R[2] * z2z2), s2 = md(R[1] * P[2] * z1z1);
    if (u1 === u2) return s1 === s2 ? jacDouble(P) : [0n, 1n, 0n];
    const h = md(u2 - u1), i = md(4n * h * h), j = md(h * i);
    const r = md(2n * (s2 - s1)), v = md(u1 * i);
    const x3 = md(r * r - j - 2n * v);
    const y3 = md(r * (v - x3) - 2n * s1 * j);
    const z3 = md((md((P[2] + R[2]) * (P[2] + R[2])) - z1z1 - z2z2) * h);
    return [x3, y3, z3];
}

function jacToAffine(P) {
    if (P[2] === 0n) return null;
    const zi = qinv(P[2]), zi2 = md(zi * zi);
    return [md(P[0] * zi2), md(P[1] * zi2 * zi)];
}

function jacMul(P, k) {
    let R = [0n, 1n, 0n];
    for (let i = BigInt(k.toString(2).length) - 1n; i >= 0n; i--) {
        R = jacDouble(R);
        if ((k >> i) & 1n) R = jacAdd(R, P);
    }
    return R;
}

function buildG1(F1, Fr, addon) {
    const n8 = 32;
    const mont = (v) => toLE((md(v) * MONT) % Q);
    const unmont = (b, o) => (fromLE(b.subarray(o, o + n8)) * F1.Rinv) % Q;
    // Uint8Array (96 B Jacobian or 64 B affine, Montgomery) -> internal
    function dec(a) {
        if (a.byteLength === 3 * n8) {
            const z = unmont(a, 2 * n8);
            return z === 0n ? [0n, 1n, 0n] : [unmont(a, 0), unmont(a, n8), z];
        }
        if (a.byteLength === 2 * n8) {
            const x = unmont(a, 0), y = unmont(a, n8);
            return x === 0n && y === 0n ? [0n, 1n, 0n] : [x, y, 1n];
        }
        throw new Error("G1: invalid point size");
    }
    function encJ(P) {
        const out = new Uint8Array(3 * n8);
        if (P[2] === 0n) { out.set(mont(1n), n8); return out; }  // (0, 1, 0)
        out.set(mont(P[0]), 0); out.set(mont(P[1]), n8); out.set(mont(P[2]), 2 * n8);
        return out;
    }
    function encA(P) {
        const out = new Uint8Array(2 * n8);
        const A = jacToAffine(P);
        if (A) { out.set(mont(A[0]), 0); out.set(mont(A[1]), n8); }
        return out;
    }
    const scalarOf = (s) => (typeof s === "bigint" ? s : fromLE(s.length > 32 ? s.subarray(0, 32) : s));
    const G1 = {
        F: F1,
        zero: encJ([0n, 1n, 0n]),
        one: encJ([1n, 2n, 1n]),
        zeroAffine: new Uint8Array(2 * n8),
        oneAffine: encA([1n, 2n, 1n]),
        add: (a, b) => encJ(jacAdd(dec(a), dec(b))),
        sub: (a, b) => { const B = dec(b); return encJ(jacAdd(dec(a), [B[0], md(-B[1]), B[2]])); },
        neg: (a) => {
            const P = dec(a);
            const N = [P[0], md(-P[1]), P[2]];
            return a.byteLength === 2 * n8 ? encA(N) : encJ(N);
        },
        double: (a) => encJ(jacDouble(dec(a))),
        eq: (a, b) => {
            const A = jacToAffine(dec(a)), B = jacToAffine(dec(b));
            return A === null || B === null ? A === B : A[0] === B[0] && A[1] === B[1];
        },
        isZero: (a) => dec(a)[2] === 0n,
        // scalar as an Fr element (Montgomery bytes)
        timesFr: (a, s) => encJ(jacMul(dec(a), Fr.toObject(s))),
        // scalar as a little-endian integer (bytes) or a BigInt
        timesScalar: (a, s) => encJ(jacMul(dec(a), scalarOf(s))),
        toAffine: (a) => encA(dec(a)),
        toJacobian: (a) => encJ(dec(a)),
        isValid: (a) => {
            const A = jacToAffine(dec(a));
            return A === null || md(A[1] * A[1]) === md(A[0] * A[0] * A[0] + G1_B);
        },
        // x||y big-endian standard form; the zero point -> 0x40 then zeros
        toRprUncompressed: (buff, o, a) => {
            const A = jacToAffine(dec(a));
            if (A === null) { buff.fill(0, o, o + 2 * n8); buff[o] = 0x40; return; }
            buff.set(toLE(A[0]).reverse(), o);
            buff.set(toLE(A[1]).reverse(), o + n8);
        },
        fromRprUncompressed: (buff, o) => {
            if (buff[o] & 0x40) return encA([0n, 1n, 0n]);
            const x = fromLE(buff.slice(o, o + n8).reverse()), y = fromLE(buff.slice(o + n8, o + 2 * n8).reverse());
            return encA([x, y, 1n]);
        },
        toRprLEM: (buff, o, a) => buff.set(encA(dec(a)), o),
        fromRprLEM: (buff, o) => new Uint8Array(buff.slice(o, o + 2 * n8)),
        toObject: (a) => { const A = jacToAffine(dec(a)); return A === null ? [0n, 1n, 0n] : [A[0], A[1], 1n]; },
        fromObject: (o) => encJ([BigInt(o[0]), BigInt(o[1]), o.length > 2 ? BigInt(o[2]) : 1n]),
        toString: (a, radix = 10) => {
            const A = jacToAffine(dec(a));
            return A === null ? "[ 0, 1, 0 ]" : `[ ${A[0].toString(radix)}, ${A[1].toString(radix)}, 1 ]`;
        },
        // [ffjs] G1.multiExpAffine(bases, scalars): bases = n x 64 B affine LEM, scalars = n x 32 B
        // standard-form LE (the reference passes Fr.batchFromMontgomery(coef), polynomial.js:1112);
        // returns a Jacobian point. Small inputs on the host, the rest on the GPU (kgs_msm).
        multiExpAffine: async (bases, scalars) => {
            const n = Math.floor(scalars.byteLength / 32);
            if (bases.byteLength < 64 * n) throw new Error("multiExpAffine: not enough bases");
            if (n <= 16) {
                let R = [0n, 1n, 0n];
                for (let i = 0; i < n; i++)
                    R = jacAdd(R, jacMul(dec(bases.subarray(64 * i, 64 * i + 64)), fromLE(scalars.subarray(32 * i, 32 * i + 32))));
                return encJ(R);
            }
            const a = addon();
            // async on a libuv thread (the bases' window tables are built there, not on the event
            // loop); the shim context's point set is per call, so its MSMs run one at a time
            const run = () => a.msmPoints(shimContext(a), bases.subarray(0, 64 * n), scalars.subarray(0, 32 * n));
            const p = shimBusy.then(run, run);
            shimBusy = p.catch(() => {});
            return encJ(dec(await p));
        },
    };
    return G1;
}

// one context of its own for the shim's MSMs (its point set is replaced by every call)
let shimCtx = null;
let shimBusy = Promise.resolve();
function shimContext(a) {
    if (!shimCtx) shimCtx = a.ctxCreate(0);
    return shimCtx;
}

// ---------------------------------------------------------------- G2 (affine / Jacobian over Fq2)
const G2_GEN = [
    [10857046999023057135944570762232829481370756359578518086990519993285655852781n,
     11559732032986387107991004021392285783925812861821192530917403151452391805634n],
    [8495653923123431417604973247489272438418190587263600148770280649306958101930n,
     4082367875863433681332203403145435568316851327593401208105741076214120093531n],
];

function buildG2(F1) {
    const n8 = 64;
    const enc = (x, o, out) => { out.set(toLE((md(x) * MONT) % Q), o); };
    function affine(P) {
        const out = new Uint8Array(2 * n8);
        enc(P[0][0], 0, out); enc(P[0][1], 32, out); enc(P[1][0], 64, out); enc(P[1][1], 96, out);
        return out;
    }
    const oneA = affine(G2_GEN);
    const oneJ = new Uint8Array(3 * n8);
    oneJ.set(oneA, 0);
    oneJ.set(toLE(MONT % Q), 2 * n8);  // z = 1 + 0u
    return {
        F: { n8 },
        one: oneJ,
        oneAffine: oneA,
        // only Jacobian points with z = 1 (the forms this shim and ptau files produce) are supported
        toAffine: (a) => {
            if (a.byteLength === 2 * n8) return new Uint8Array(a);
            const z0 = fromLE(a.subarray(2 * n8, 2 * n8 + 32)), z1 = fromLE(a.subarray(2 * n8 + 32, 3 * n8));
            if (z0 === 0n && z1 === 0n) return new Uint8Array(2 * n8);
            if (z0 !== MONT % Q || z1 !== 0n) throw new Error("G2.toAffine: only z = 1 points are supported by the shim");
            return new Uint8Array(a.subarray(0, 2 * n8));
        },
        toRprLEM: (buff, o, a) => buff.set(a.byteLength === 2 * n8 ? a : a.subarray(0, 2 * n8), o),
        fromRprLEM: (buff, o) => new Uint8Array(buff.slice(o, o + 2 * n8)),
    };
}

function buildBn128() {
    const Fr = new Field(R);
    const F1 = new Field(Q);
    // Fr.w[k]: primitive 2^k-th roots, nqr = 5, s = 28
    Fr.s = 28;
    Fr.w = new Array(29);
    let w = modpow(5n, (R - 1n) >> 28n, R);
    for (let k = 28; k >= 0; k--) { Fr.w[k] = Fr.e(w); w = (w * w) % R; }
    const addon = () => require("./backend.js").load();
    // [ffjs] Fr batch members (grandsum.js:41 batchInverse, polynomial.js:34,152,160 fft / ifft,
    // polynomial.js:1112 batchFromMontgomery, prover.js:147-148 batchToMontgomery)
    async function frOp(op, buff) {
        if (Array.isArray(buff)) {  // an array of elements in, an array of elements out
            const packed = new Uint8Array(32 * buff.length);
            buff.forEach((e, i) => packed.set(e, 32 * i));
            const out = await frOp(op, packed);
            return buff.map((_, i) => out.slice(32 * i, 32 * i + 32));
        }
        const flat = contiguous(buff);
        if (flat.byteLength % 32) throw new Error("Fr: the buffer must hold 32-byte elements");
        let out;
        if (flat.byteLength === 0) {
            out = new Uint8Array(0);
        } else {
            const a = addon();
            out = await a.frOp(shimContext(a), op, flat);
        }
        if (!(buff instanceof BigBuffer)) return out;
        const bb = new BigBuffer(out.byteLength);
        bb.set(out, 0);
        return bb;
    }
    Fr.batchToMontgomery = (buff) => frOp(0, buff);
    Fr.batchFromMontgomery = (buff) => frOp(1, buff);
    Fr.batchInverse = (buff) => frOp(2, buff);  // zero elements stay zero
    Fr.fft = (buff) => frOp(3, buff);           // 2^k elements, natural order, w = Fr.w[k]
    Fr.ifft = (buff) => frOp(4, buff);          // includes the 1/2^k
    const G1 = buildG1(F1, Fr, addon);
    const G2 = buildG2(F1);
    return {
        name: "bn128",
        Fr,
        F1,
        G1,
        G2,
        // [ffjs] curve.pairingEq(a1, b1, a2, b2, ...): prod e(a_k, b_k) == 1, native optimal-ate pairing
        pairingEq: async (...args) => {
            if (args.length % 2) throw new Error("pairingEq: expected (G1, G2) pairs");
            const n = args.length / 2;
            const g1 = new Uint8Array(64 * n), g2 = new Uint8Array(128 * n);
            for (let k = 0; k < n; k++) {
                g1.set(G1.toAffine(args[2 * k]), 64 * k);
                g2.set(G2.toAffine(args[2 * k + 1]), 128 * k);
            }
            return addon().pairingEq(g1, g2);
        },
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
