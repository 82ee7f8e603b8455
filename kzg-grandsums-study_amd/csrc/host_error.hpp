// Error type and per-thread last-error message of the C-ABI (include/kgs.h: every entry point
// returns a KGS_E_* code, kgs_last_error() the message of the calling thread's last failure).
// Host-only; shared by the prover (prover.cpp) and the host-only units (ptau_io.cpp, verifier.cpp).
#pragma once
#include <stdexcept>
#include <string>

namespace kgs {

struct KgsError : std::runtime_error {
  int code;
  KgsError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// the calling thread's last-error slot (defined in ptau_io.cpp)
std::string& kgs_errbuf();

inline int kgs_fail(const KgsError& e) {
  kgs_errbuf() = e.what();
  return e.code;
}

}  // namespace kgs
