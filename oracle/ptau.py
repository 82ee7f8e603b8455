"""ptau binfile reader / synthetic writer for the CPU ORACLE — test infrastructure only.

Restates `@iden3/binfileutils@0.0.11` `readBinFile(fn, "ptau", 1, ...)` and the reference's
`readPTauHeader` (src/ptau_utils.js:3-24):

    "ptau" | u32 version | u32 nSections | { u32 id | u64 size | payload }*
    section 1: u32 n8 | q (n8 B LE) | u32 power | u32 ceremonyPower
    section 2: tauG1, 2^(power+1)-1 affine G1 points, 64 B LEM each
    section 3: tauG2, 128 B LEM each ([tau]_2 is the point at byte offset 128,
               src/grandsum/mset_eq_kzg_verifier.js:18-19)

The synthetic writer produces a file with the SAME layout from a known tau; its
section 3 is truncated to the first two G2 points (all the reference ever reads). Knowing tau lets
tests check every commitment in closed form: MSM(SRS, c) == (sum c_i tau^i)·G1.
"""
import struct

from . import bn254 as bn


def read_sections(path):
    with open(path, "rb") as fh:
        data = fh.read()
    if data[:4] != b"ptau":
        raise ValueError(f"{path}: Invalid File format")
    version, nsec = struct.unpack_from("<II", data, 4)
    if version > 1:
        raise ValueError(f"{path}: Invalid Version")
    pos = 12
    sections = {}
    for _ in range(nsec):
        sid, size = struct.unpack_from("<IQ", data, pos)
        pos += 12
        sections.setdefault(sid, []).append((pos, size))
        pos += size
    return data, sections


def read_header(data, sections):
    """src/ptau_utils.js:3-24 -> (q, power, ceremonyPower)."""
    if 1 not in sections:
        raise ValueError("File has no  header")
    if len(sections[1]) > 1:
        raise ValueError("File has more than one header")
    p, size = sections[1][0]
    n8 = struct.unpack_from("<I", data, p)[0]
    q = int.from_bytes(data[p + 4:p + 4 + n8], "little")
    power, cpower = struct.unpack_from("<II", data, p + 4 + n8)
    if 4 + n8 + 8 != size:
        raise ValueError("Invalid PTau header size")
    if q != bn.Q or n8 != 32:
        raise ValueError("ptau curve is not bn128")
    return q, power, cpower


class PTau:
    """In-memory view of the parts of a ptau file the provers/verifiers read."""

    def __init__(self, path):
        data, sections = read_sections(path)
        self.q, self.power, self.ceremony_power = read_header(data, sections)
        p2, s2 = sections[2][0]
        self.g1_bytes = data[p2:p2 + s2]
        p3, s3 = sections[3][0]
        self.g2_bytes = data[p3:p3 + s3]
        self.tau = None
        self._g1_cache = {}

    def g1_point(self, i):
        if i not in self._g1_cache:
            self._g1_cache[i] = bn.g1_from_lem(self.g1_bytes[64 * i:64 * i + 64])
        return self._g1_cache[i]

    def tau_g2(self):
        return bn.g2_from_lem(self.g2_bytes[128:256])


def _fixed_base_table(base, bits=256, w=8):
    table = []
    cur = base
    for _ in range((bits + w - 1) // w):
        row = [None] * (1 << w)
        acc = None
        for k in range(1, 1 << w):
            acc = bn.g1_add(acc, cur)
            row[k] = acc
        table.append(row)
        # cur <<= w
        for _ in range(w):
            cur = bn.g1_add(cur, cur)
    return table


def _batch_to_affine(jacs):
    zs = [P[2] for P in jacs]
    pref = []
    acc = 1
    for z in zs:
        pref.append(acc)
        acc = acc * (z if z else 1) % bn.Q
    inv = bn.fq_inv(acc)
    out = [None] * len(jacs)
    for i in range(len(jacs) - 1, -1, -1):
        z = zs[i]
        if z == 0:
            continue
        zi = inv * pref[i] % bn.Q
        inv = inv * z % bn.Q
        X, Y, _ = jacs[i]
        zi2 = zi * zi % bn.Q
        out[i] = (X * zi2 % bn.Q, Y * zi2 * zi % bn.Q)
    return out


def synth_g1_powers(tau, count):
    """[tau^i]_1 for i < count (affine)."""
    w = 8
    table = _fixed_base_table(bn.G1_GEN, 256, w)
    jac = []
    t = 1
    for _ in range(count):
        acc = (1, 1, 0)
        k = t
        j = 0
        while k:
            d = k & 0xFF
            if d:
                acc = bn._jac_add(acc, bn._to_jac(table[j][d]))
            k >>= w
            j += 1
        jac.append(acc)
        t = t * tau % bn.R
    return _batch_to_affine(jac)


def write_synthetic_ptau(path, power, tau, g1_points=None):
    """Write a ptau with sections 1-3 for a known tau (section 3 truncated to 2 G2 points)."""
    n1 = (1 << (power + 1)) - 1
    if g1_points is None:
        g1_points = synth_g1_powers(tau, n1)
    sec1 = struct.pack("<I", 32) + bn.Q.to_bytes(32, "little") + struct.pack("<II", power, power)
    sec2 = b"".join(bn.g1_to_lem(p) for p in g1_points[:n1])
    sec3 = bn.g2_to_lem(bn.G2_GEN) + bn.g2_to_lem(bn.g2_mul(bn.G2_GEN, tau))
    with open(path, "wb") as fh:
        fh.write(b"ptau" + struct.pack("<II", 1, 3))
        for sid, payload in ((1, sec1), (2, sec2), (3, sec3)):
            fh.write(struct.pack("<IQ", sid, len(payload)))
            fh.write(payload)


def bench_tau():
    """tau = keccak256("kgs-bench-tau") mod r."""
    from .keccak import keccak256
    return int.from_bytes(keccak256(b"kgs-bench-tau"), "big") % bn.R
