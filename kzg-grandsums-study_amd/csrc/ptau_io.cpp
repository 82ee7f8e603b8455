// Host-only ptau header parsing and the C-ABI entry points that read ptau files without a GPU
// (kgs_ptau_power, kgs_ptau_read_tau_g2), plus the library's last-error slot. The file is
// untrusted input: every offset and size read from it is checked against the file size before it
// is used (tests/native/host_check.cpp runs these paths under ASan/UBSan on malformed files).
// Format: "ptau", u32 version, u32 nsections, then nsections x (u32 id, u64 size, payload);
// section 1 = header (u32 n8, q (n8 bytes), u32 power, u32 ceremonyPower), section 2 = tauG1,
// section 3 = tauG2 (src/ptau_utils.js:3-24; @iden3/binfileutils readBinFile).
#include "ptau_io.hpp"

#include <string.h>
#include <sys/types.h>

#include <memory>
#include <string>

#include "../../include/kgs.h"
#include "host_error.hpp"
#include "host_field.hpp"

namespace kgs {

std::string& kgs_errbuf() {
  static thread_local std::string err;
  return err;
}

PtauInfo read_ptau_header(FILE* f, const char* path) {
  PtauInfo info;
  const std::string p(path ? path : "");
  if (fseeko(f, 0, SEEK_END) != 0) throw KgsError(KGS_E_IO, p + ": cannot seek");
  const off_t fend = ftello(f);
  if (fend < 0) throw KgsError(KGS_E_IO, p + ": cannot tell size");
  const uint64_t fsize = (uint64_t)fend;
  info.file_size = fsize;
  char magic[4];
  uint32_t ver = 0, nsec = 0;
  if (fseeko(f, 0, SEEK_SET) != 0 || fread(magic, 1, 4, f) != 4 || memcmp(magic, "ptau", 4) != 0)
    throw KgsError(KGS_E_IO, p + ": Invalid File format");
  if (fread(&ver, 4, 1, f) != 1 || fread(&nsec, 4, 1, f) != 1) throw KgsError(KGS_E_IO, p + ": truncated ptau");
  if (ver > 1) throw KgsError(KGS_E_IO, p + ": Invalid Version");
  if ((uint64_t)nsec > (fsize - 12) / 12) throw KgsError(KGS_E_IO, p + ": truncated ptau section table");
  uint64_t pos = 12;
  int nheaders = 0;
  uint64_t s1_pos = 0, s1_size = 0;
  for (uint32_t s = 0; s < nsec; s++) {
    uint32_t id = 0;
    uint64_t size = 0;
    if (pos > fsize || fsize - pos < 12) throw KgsError(KGS_E_IO, p + ": truncated ptau section table");
    if (fseeko(f, (off_t)pos, SEEK_SET) || fread(&id, 4, 1, f) != 1 || fread(&size, 8, 1, f) != 1)
      throw KgsError(KGS_E_IO, p + ": truncated ptau section table");
    pos += 12;
    if (size > fsize - pos) throw KgsError(KGS_E_IO, p + ": section extends past the end of the file");
    if (id == 1) {
      nheaders++;
      s1_pos = pos;
      s1_size = size;
    } else if (id == 2 && !info.s2_size) {
      info.s2_pos = pos;
      info.s2_size = size;
    } else if (id == 3 && !info.s3_size) {
      info.s3_pos = pos;
      info.s3_size = size;
    }
    pos += size;
  }
  if (!nheaders) throw KgsError(KGS_E_IO, p + ": File has no  header");
  if (nheaders > 1) throw KgsError(KGS_E_IO, p + ": File has more than one header");
  if (s1_size != 4 + 32 + 8) throw KgsError(KGS_E_IO, p + ": Invalid PTau header size");
  uint32_t n8 = 0;
  uint8_t q[32];
  uint32_t pw[2] = {0, 0};
  if (fseeko(f, (off_t)s1_pos, SEEK_SET) || fread(&n8, 4, 1, f) != 1 || n8 != 32 || fread(q, 1, 32, f) != 32 ||
      fread(pw, 4, 2, f) != 2)
    throw KgsError(KGS_E_IO, p + ": Invalid size");
  if (memcmp(q, host::FQ_MOD.p, 32) != 0) throw KgsError(KGS_E_IO, p + ": ptau curve is not bn128");
  if (pw[0] < 1 || pw[0] > 63) throw KgsError(KGS_E_IO, p + ": Invalid power");
  info.power = (int)pw[0];
  info.ceremony = (int)pw[1];
  return info;
}

}  // namespace kgs

using namespace kgs;

extern "C" {

const char* kgs_last_error(void) { return kgs_errbuf().c_str(); }
const char* kgs_version(void) { return "kgs-mi355x 0.2 (gfx950)"; }

int kgs_ptau_power(const char* path, int* power) {
  try {
    if (!path || !power) throw KgsError(KGS_E_ARG, "NULL argument");
    FILE* f = fopen(path, "rb");
    if (!f) throw KgsError(KGS_E_IO, std::string("cannot open ") + path);
    std::unique_ptr<FILE, int (*)(FILE*)> guard(f, fclose);
    *power = read_ptau_header(f, path).power;
    return KGS_OK;
  } catch (const KgsError& e) {
    return kgs_fail(e);
  } catch (const std::exception& e) {
    kgs_errbuf() = e.what();
    return KGS_E_IO;
  }
}

int kgs_ptau_read_tau_g2(const char* path, uint8_t out128[128]) {
  try {
    if (!path || !out128) throw KgsError(KGS_E_ARG, "NULL argument");
    FILE* f = fopen(path, "rb");
    if (!f) throw KgsError(KGS_E_IO, std::string("cannot open ") + path);
    std::unique_ptr<FILE, int (*)(FILE*)> guard(f, fclose);
    PtauInfo info = read_ptau_header(f, path);
    if (info.s3_size < 256) throw KgsError(KGS_E_IO, "tauG2 section too small");
    if (fseeko(f, (off_t)(info.s3_pos + 128), SEEK_SET) || fread(out128, 1, 128, f) != 128)
      throw KgsError(KGS_E_IO, "cannot read [tau]_2");
    return KGS_OK;
  } catch (const KgsError& e) {
    return kgs_fail(e);
  } catch (const std::exception& e) {
    kgs_errbuf() = e.what();
    return KGS_E_IO;
  }
}

}  // extern "C"
