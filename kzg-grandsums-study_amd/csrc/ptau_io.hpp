// ptau (iden3 binfileutils layout) header parsing — host-only, the untrusted-input side of the SRS
// load (readBinFile + readPTauHeader, src/ptau_utils.js:3-24). Built with the library and, for the
// CPU sanitizer tests, under ASan/UBSan (tests/native).
#pragma once
#include <stdint.h>
#include <stdio.h>

namespace kgs {

struct PtauInfo {
  int power = 0, ceremony = 0;
  uint64_t file_size = 0;
  uint64_t s2_pos = 0, s2_size = 0, s3_pos = 0, s3_size = 0;  // 0 size: section absent
};

// Validates the whole section table against the file size and the bn128 header; throws KgsError
// (KGS_E_IO) with binfileutils' messages where it has one.
PtauInfo read_ptau_header(FILE* f, const char* path);

}  // namespace kgs
