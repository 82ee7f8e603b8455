// The drop-in provers' log channel: the reference logs through logplease at INFO (logger.js:1-5,
// used by src/grandsum/mset_eq_kzg_prover.js:13-140,164-412 and its grand-product twin). Here the
// level comes from KGS_LOG_LEVEL (DEBUG, INFO, WARN, ERROR, NONE; default WARN, so a proof prints
// only the reference's warnings unless asked), and setLogger() plugs in the caller's own logger
// object (e.g. the reference's logplease instance: every line then goes through it, with its
// formatting and level). Message texts are the reference's; the built-in sink writes to stderr.
const LEVELS = { DEBUG: 0, INFO: 1, WARN: 2, ERROR: 3, NONE: 4 };

function parseLevel(name) {
    const k = String(name || "").toUpperCase();
    return Object.prototype.hasOwnProperty.call(LEVELS, k) ? LEVELS[k] : LEVELS.WARN;
}

let level = parseLevel(process.env.KGS_LOG_LEVEL);
let sink = null;

function emit(name, args) {
    if (sink) {
        const fn = sink[name.toLowerCase()];
        if (typeof fn === "function") fn.apply(sink, args);
        return;
    }
    if (LEVELS[name] >= level) console.error(`[${name}]`, ...args);  // stderr: stdout stays the caller's
}

module.exports = {
    debug: (...a) => emit("DEBUG", a),
    info: (...a) => emit("INFO", a),
    warn: (...a) => emit("WARN", a),
    error: (...a) => emit("ERROR", a),
    // true when a line of this level reaches an output (an injected logger decides for itself)
    enabled: (name) => sink !== null || LEVELS[String(name).toUpperCase()] >= level,
    setLogLevel: (name) => { level = parseLevel(name); },
    setLogger: (l) => { sink = l || null; },
};
