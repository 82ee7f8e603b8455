// [ffjs] Scalar: arbitrary-precision integers as BigInt. The reference uses fromRprBE for the
// transcript challenge (src/Keccak256Transcript.js:50) and lt(fromRprLE(x), Fr.p) for the
// verifier's field-membership check (src/grandsum/mset_eq_kzg_verifier.js:195,
// src/grandproduct/mset_eq_kzg_verifier.js:187); the rest is the obvious companion set.
function bytesOf(buff, o, n8) {
    const b = buff instanceof Uint8Array ? buff : new Uint8Array(buff.buffer || buff, buff.byteOffset || 0);
    o = o || 0;
    n8 = n8 === undefined ? b.byteLength - o : n8;
    return b.subarray(o, o + n8);
}

const Scalar = {
    e: (a, base) => (typeof a === "string" && base === 16 && !a.startsWith("0x") ? BigInt("0x" + a) : BigInt(a)),
    fromString: (s, radix = 10) => (radix === 16 ? BigInt("0x" + s.replace(/^0x/, "")) : BigInt(s)),
    toString: (a, radix = 10) => BigInt(a).toString(radix),
    fromRprLE(buff, o, n8) {
        const b = bytesOf(buff, o, n8);
        let x = 0n;
        for (let i = b.length - 1; i >= 0; i--) x = (x << 8n) | BigInt(b[i]);
        return x;
    },
    fromRprBE(buff, o, n8) {
        const b = bytesOf(buff, o, n8);
        let x = 0n;
        for (let i = 0; i < b.length; i++) x = (x << 8n) | BigInt(b[i]);
        return x;
    },
    toRprLE(buff, o, a, n8) {
        let x = BigInt(a);
        for (let i = 0; i < n8; i++) { buff[o + i] = Number(x & 0xffn); x >>= 8n; }
    },
    toRprBE(buff, o, a, n8) {
        let x = BigInt(a);
        for (let i = n8 - 1; i >= 0; i--) { buff[o + i] = Number(x & 0xffn); x >>= 8n; }
    },
    lt: (a, b) => BigInt(a) < BigInt(b),
    leq: (a, b) => BigInt(a) <= BigInt(b),
    gt: (a, b) => BigInt(a) > BigInt(b),
    geq: (a, b) => BigInt(a) >= BigInt(b),
    eq: (a, b) => BigInt(a) === BigInt(b),
    isZero: (a) => BigInt(a) === 0n,
    bitLength: (a) => (BigInt(a) === 0n ? 0 : BigInt(a).toString(2).length),
};

module.exports = { Scalar };
