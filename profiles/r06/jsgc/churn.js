// CPU-only reproduction of the JS prover's garbage (round 6, DESIGN.md §13 "The boundary"): inputs
// made up front; per simulated proof (every 15 ms) two 32 MiB input buffers lose their last
// reference (the reference replaces Evaluations.eval by the Montgomery copy, prover.js:147-148) and
// two 32 MiB outputs appear. Run: node --trace-gc churn.js [KEEP=1 keeps the inputs alive].
const n = 1 << 20, N = 15;
const f = new Uint8Array(32 * n);
for (let i = 0; i < f.length; i += 4096) f[i] = 1;
const lat = Array.from({ length: N }, () => [f.slice(), f.slice()]);
const keep = [];
let i = 0;
function step() {
    if (i >= N) { console.log("done"); process.exit(0); }
    const [a, b] = lat[i];
    if (!process.env.KEEP) lat[i] = null;
    const o1 = new Uint8Array(32 * n), o2 = new Uint8Array(32 * n);
    o1[0] = a[0]; o2[0] = b[0];
    keep.push(o1, o2);
    i++;
    setTimeout(step, 15);
}
setTimeout(step, 50);
