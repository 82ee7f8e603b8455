// Keccak-256 Fiat-Shamir transcript exactly as src/Keccak256Transcript.js:7-53: commitments enter
// as G1.toRprUncompressed (64 B, big-endian standard x||y), scalars as Fr.toRprBE (32 B); the
// challenge is the big-endian hash reduced mod r; the buffer is cumulative (never reset).
#pragma once
#include <vector>

#include "host_field.hpp"
#include "keccak.hpp"

namespace kgs {
namespace host {

struct Transcript {
  std::vector<uint8_t> buf;
  void add_commitment(const uint8_t lem[64]) {
    uint8_t rpr[64];
    host::g1_lem_to_rpr_uncompressed(lem, rpr);
    buf.insert(buf.end(), rpr, rpr + 64);
  }
  void add_scalar(const Fr& s) {
    uint8_t be[32];
    s.to_be_std(be);
    buf.insert(buf.end(), be, be + 32);
  }
  Fr challenge() const {
    uint8_t h[32];
    host::keccak256(buf.data(), buf.size(), h);
    return Fr::from_be_reduce(h);
  }
};

}  // namespace host
}  // namespace kgs
