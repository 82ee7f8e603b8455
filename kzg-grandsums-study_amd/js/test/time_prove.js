// Times the JavaScript drop-in prover end to end (module call -> N-API -> libkgs -> proof object),
// as a reference user would call it: node time_prove.js PTAU NBITS [PROOFS] [CONCURRENCY].
// Inputs are random standard-form field elements (< 2^253 < r) in Uint8Arrays, T = F rotated by one
// element, prepared before the timed regions (the prover overwrites them with Montgomery form, so
// every proof gets its own copy).
//  * latency: one proof at a time, back to back (inputs prepared beforehand): best, median and spread
//    of PROOFS; under node --expose-gc also a second series in which the caller runs gc() before each
//    timed call (latency_ms_caller_gc_between);
//  * concurrent throughput: PROOFS * CONCURRENCY proofs issued as CONCURRENCY independent chains of
//    awaited prover() calls (the reference API is async; independent calls run on the backend's
//    context pool), wall clock of the whole batch.
// Prints one JSON line: {nbits, proofs, ms_per_proof, proofs_per_s, concurrency, concurrent_proofs,
// concurrent_proofs_per_s, pool, verified}.
const crypto = require("crypto");
const { getCurveFromName, Evaluations, mset_eq_kzg_grandsum_prover, mset_eq_kzg_grandsum_verifier } = require("../index");
const { poolInfo, diag } = require("../src/backend");

(async () => {
    const [ptau, nbArg, nArg, cArg] = process.argv.slice(2);
    const nBits = parseInt(nbArg, 10), proofs = parseInt(nArg || "5", 10), conc = parseInt(cArg || "0", 10);
    const n = 2 ** nBits;
    const curve = await getCurveFromName("bn128");
    const f = new Uint8Array(crypto.randomBytes(32 * n));
    for (let i = 0; i < n; i++) f[32 * i + 31] &= 0x1f;  // < 2^253
    const t = new Uint8Array(32 * n);
    t.set(f.subarray(0, 32 * (n - 1)), 32);
    t.set(f.subarray(32 * (n - 1)), 0);
    const mk = () => [new Evaluations(f.slice(), curve), new Evaluations(t.slice(), curve)];
    let [F, T] = mk();
    let proof = await mset_eq_kzg_grandsum_prover(ptau, F, T);  // warm: context, SRS, buffers
    let best = Infinity, bestDiag = null;
    const all = [], diags = [], calls = [];
    // fresh standard-form inputs per proof (the prover overwrites them with Montgomery form), all made
    // before the timed loop so the proofs run back to back, as the Python latency probe's do
    const lat = Array.from({ length: proofs }, mk);
    for (let i = 0; i < proofs; i++) {
        [F, T] = lat[i];
        const t0 = process.hrtime.bigint();
        proof = await mset_eq_kzg_grandsum_prover(ptau, F, T);
        const ms = Number(process.hrtime.bigint() - t0) / 1e6;
        all.push(+ms.toFixed(3));
        diags.push([+diag.execMs.toFixed(3)].concat(diag.timing.map(x => +x.toFixed(3))));
        calls.push([+diag.callMs.toFixed(3)].concat(diag.waitMs.map(x => +x.toFixed(3))));
        if (ms < best) {
            best = ms;
            bestDiag = { exec_ms: +diag.execMs.toFixed(3), libkgs_timing_ms: diag.timing.map(x => +x.toFixed(3)) };
        }
    }
    const stats = xs => {
        const s = xs.slice().sort((a, b) => a - b), m = s.length >> 1;
        return { median: +(s.length % 2 ? s[m] : (s[m - 1] + s[m]) / 2).toFixed(3), min: s[0], max: s[s.length - 1],
                 samples: s.length };
    };
    const verified = await mset_eq_kzg_grandsum_verifier(ptau, proof, nBits);
    const out = { nbits: nBits, proofs, ms_per_proof: +best.toFixed(3), proofs_per_s: +(1000 / best).toFixed(3), verified,
                  latency_ms: stats(all), best_inside_libkgs: bestDiag,
                  eager_gc: process.env.KGS_JS_EAGER_GC || null };
    // a caller that collects its own garbage between proofs (node --expose-gc; gc() outside the timed
    // call): the previous proof's replaced input buffers are freed before the next call starts
    if (typeof global.gc === "function" && !process.env.KGS_JS_EAGER_GC) {
        const lat2 = Array.from({ length: proofs }, mk), all2 = [];
        for (let i = 0; i < proofs; i++) {
            [F, T] = lat2[i];
            lat2[i] = null;
            global.gc();
            const t0 = process.hrtime.bigint();
            proof = await mset_eq_kzg_grandsum_prover(ptau, F, T);
            all2.push(+(Number(process.hrtime.bigint() - t0) / 1e6).toFixed(3));
        }
        out.latency_ms_caller_gc_between = stats(all2);
    }
    if (process.env.KGS_JS_TIME_ALL) {  // every latency sample: [exec_ms, libkgs timing...] each
        out.all_ms = all;
        out.all_inside_libkgs = diags;
        out.all_native_call = calls;  // [native call wall ms, queue -> worker ms, worker -> completion ms]
    }
    if (conc > 0) {
        // warm every context of the pool (SRS tables are shared per device; buffers are per context)
        await Promise.all(Array.from({ length: conc }, () => { const [a, b] = mk(); return mset_eq_kzg_grandsum_prover(ptau, a, b); }));
        const total = proofs * conc;
        const inputs = Array.from({ length: total }, mk);
        let next = 0;
        const results = [];
        const chain = async () => {
            while (next < total) {
                const [a, b] = inputs[next++];
                results.push(await mset_eq_kzg_grandsum_prover(ptau, a, b));
            }
        };
        const t0 = process.hrtime.bigint();
        await Promise.all(Array.from({ length: conc }, chain));
        const s = Number(process.hrtime.bigint() - t0) / 1e9;
        // every proof of the batch is of the same statement: all must be identical to the verified one
        const hx = p => Buffer.from(p.commitments.Wxi).toString("hex") + Buffer.from(p.evaluations.sxiw).toString("hex");
        out.concurrency = conc;
        out.concurrent_proofs = total;
        out.concurrent_proofs_per_s = +(total / s).toFixed(3);
        out.concurrent_all_identical = results.every(p => hx(p) === hx(proof));
        out.pool = poolInfo();
    }
    console.log(JSON.stringify(out));
    process.exit(0);
})().catch(e => { console.error(e); process.exit(1); });
