// [ffjs] BigBuffer: a byte buffer larger than one typed array may be, as pages of 2^30 bytes. The
// reference allocates one for the 2n-point PTau slice (src/grandsum/mset_eq_kzg_prover.js:83) and
// for large polynomials (src/polynomial/polynomial.js:40-44); Evaluations.fromPolynomial hands one
// to Fr.fft (src/polynomial/evaluations.js:12-21). Members the reference touches: byteLength,
// set(src, offset), slice(from, to), and the pages in `buffers`.
const PAGE = 1 << 30;

class BigBuffer {
    constructor(size) {
        this.byteLength = size;
        this.buffers = [];
        for (let left = size; left > 0; left -= PAGE) this.buffers.push(new Uint8Array(Math.min(left, PAGE)));
    }

    // copy of [from, to): a Uint8Array when it fits one page, a BigBuffer otherwise
    slice(from = 0, to = this.byteLength) {
        if (from < 0) from = Math.max(this.byteLength + from, 0);
        if (to < 0) to = Math.max(this.byteLength + to, 0);
        to = Math.min(to, this.byteLength);
        const len = Math.max(to - from, 0);
        const out = len <= PAGE ? new Uint8Array(len) : new BigBuffer(len);
        let o = 0;
        while (o < len) {
            const p = Math.floor((from + o) / PAGE), off = (from + o) % PAGE;
            const n = Math.min(PAGE - off, len - o);
            out.set(this.buffers[p].subarray(off, off + n), o);
            o += n;
        }
        return out;
    }

    // copy src (Uint8Array, Buffer or BigBuffer) to byte offset `offset`
    set(src, offset = 0) {
        if (src instanceof BigBuffer) {
            let o = 0;
            for (const b of src.buffers) { this.set(b, offset + o); o += b.byteLength; }
            return;
        }
        if (offset + src.byteLength > this.byteLength) throw new RangeError("BigBuffer.set: source does not fit");
        let o = 0;
        while (o < src.byteLength) {
            const p = Math.floor((offset + o) / PAGE), off = (offset + o) % PAGE;
            const n = Math.min(PAGE - off, src.byteLength - o);
            this.buffers[p].set(src.subarray(o, o + n), off);
            o += n;
        }
    }
}

// a contiguous Uint8Array view of a buffer the native side can take (BigBuffers are flattened)
function contiguous(buf) {
    if (buf instanceof BigBuffer) {
        if (buf.buffers.length === 1) return buf.buffers[0];
        const out = new Uint8Array(buf.byteLength);  // throws past the engine's typed-array limit
        let o = 0;
        for (const b of buf.buffers) { out.set(b, o); o += b.byteLength; }
        return out;
    }
    return buf;
}

module.exports = { BigBuffer, contiguous, PAGE };
