// Host-side sanitizer driver (TEST INFRASTRUCTURE): links the product's host-only units that parse
// untrusted bytes — ptau_io.cpp (ptau header / section table, kgs_ptau_power, kgs_ptau_read_tau_g2)
// and verifier.cpp (+ host_field.hpp / host_pairing.hpp: kgs_verify on proof bytes) — built with
// -fsanitize=address,undefined by tests/native/Makefile. tests/test_host_sanitizers.py runs it on
// malformed ptau files and proofs; any ASan/UBSan report aborts with a non-zero exit.
//
//   host_check ptau FILE                         -> "power <rc> <power>" and "g2 <rc> <hex>"
//   host_check verify KIND NBITS NPOLS SEL PTAU PROOF.bin
//                                                -> "verify <rc>" (PROOF.bin = commitments || evaluations,
//                                                   exactly kgs_proof_shape bytes, else "shape-mismatch")
//   host_check fuzz SEED ITERS PTAU              -> random shapes and bytes through kgs_verify and
//                                                   mutated copies of PTAU through the header parser
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

#include "../../include/kgs.h"

static std::vector<uint8_t> slurp(const char* path) {
  std::vector<uint8_t> d;
  FILE* f = fopen(path, "rb");
  if (!f) return d;
  uint8_t buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) d.insert(d.end(), buf, buf + n);
  fclose(f);
  return d;
}

static int cmd_ptau(const char* path) {
  int power = -1;
  int rc = kgs_ptau_power(path, &power);
  printf("power %d %d\n", rc, rc == 0 ? power : -1);
  uint8_t g2[128];
  rc = kgs_ptau_read_tau_g2(path, g2);
  printf("g2 %d ", rc);
  if (rc == 0)
    for (int i = 0; i < 128; i++) printf("%02x", g2[i]);
  printf("\n");
  return 0;
}

static int cmd_verify(int kind, int nbits, int npols, int sel, const char* ptau, const char* proof) {
  int nc = 0, ne = 0;
  kgs_proof_shape(kind, npols, sel, &nc, &ne);
  std::vector<uint8_t> d = slurp(proof);
  if (nc < 0 || ne < 0 || d.size() != (size_t)nc * 64 + (size_t)ne * 32) {
    printf("shape-mismatch\n");
    return 0;
  }
  int rc = kgs_verify_ptau(kind, ptau, nbits, npols, sel, d.data(), d.data() + (size_t)nc * 64);
  printf("verify %d\n", rc);
  return 0;
}

static int cmd_fuzz(unsigned seed, int iters, const char* ptau) {
  std::mt19937_64 rng(seed);
  std::vector<uint8_t> orig = slurp(ptau);
  uint8_t g2[128];
  if (kgs_ptau_read_tau_g2(ptau, g2) != 0) {
    printf("bad base ptau\n");
    return 1;
  }
  const std::string tmp = std::string(ptau) + ".fuzz" + std::to_string(seed);
  int accepted = 0, parsed = 0;
  for (int it = 0; it < iters; it++) {
    // 1. verifier on random shapes (including out-of-range ones) and random / structured bytes
    const int kind = (int)(rng() % 3) - (rng() % 8 == 0);
    const int nbits = (int)(rng() % 34) - 2;
    const int npols = (int)(rng() % 20) - 1;
    const int sel = (int)(rng() % 2);
    int nc = 0, ne = 0;
    kgs_proof_shape(kind, npols > 0 ? npols : 1, sel, &nc, &ne);
    std::vector<uint8_t> com((size_t)nc * 64), ev((size_t)ne * 32);
    for (auto& b : com) b = (uint8_t)rng();
    for (auto& b : ev) b = (uint8_t)rng();
    if (rng() % 2)  // infinity commitments and tiny evaluations: valid encodings, wrong proof
      for (size_t i = 0; i < com.size(); i++) com[i] = rng() % 3 ? 0 : com[i];
    if (rng() % 2)
      for (size_t i = 0; i < ev.size(); i++) ev[i] = (i % 32) < 30 ? ev[i] : 0;
    const int rc = kgs_verify(kind, nbits, npols > 0 ? npols : 1, sel, com.data(), ev.data(), rng() % 4 ? g2 : com.data());
    if (rc == 1) accepted++;
    // 2. header parser on a mutated copy of the ptau
    std::vector<uint8_t> d = orig;
    const int muts = 1 + (int)(rng() % 4);
    for (int m = 0; m < muts; m++) {
      switch (rng() % 4) {
        case 0:  // truncate
          d.resize(d.empty() ? 0 : rng() % d.size());
          break;
        case 1:  // random byte in the first 128 (magic, version, section table, header)
          if (!d.empty()) d[rng() % (d.size() < 128 ? d.size() : 128)] = (uint8_t)rng();
          break;
        case 2: {  // overwrite a 64-bit word of the section table with a huge / small value
          const size_t off = 12 + 12 * (rng() % 4) + 4;
          const uint64_t v = rng() % 2 ? ~0ull - (rng() % 64) : rng() % 512;
          if (off + 8 <= d.size()) memcpy(&d[off], &v, 8);
          break;
        }
        default:  // random byte anywhere
          if (!d.empty()) d[rng() % d.size()] = (uint8_t)rng();
      }
    }
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) return 1;
    if (!d.empty()) fwrite(d.data(), 1, d.size(), f);
    fclose(f);
    int power = 0;
    if (kgs_ptau_power(tmp.c_str(), &power) == 0) parsed++;
    uint8_t t2[128];
    kgs_ptau_read_tau_g2(tmp.c_str(), t2);
  }
  remove(tmp.c_str());
  printf("fuzz done iters %d accepted %d parsed %d\n", iters, accepted, parsed);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 3 && !strcmp(argv[1], "ptau")) return cmd_ptau(argv[2]);
  if (argc >= 8 && !strcmp(argv[1], "verify"))
    return cmd_verify(atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), argv[6], argv[7]);
  if (argc >= 5 && !strcmp(argv[1], "fuzz")) return cmd_fuzz((unsigned)atoi(argv[2]), atoi(argv[3]), argv[4]);
  fprintf(stderr, "usage: host_check ptau FILE | verify KIND NBITS NPOLS SEL PTAU PROOF | fuzz SEED ITERS PTAU\n");
  return 2;
}
