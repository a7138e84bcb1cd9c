// op_build_info (include/openpose_hip.h): the digest of the sources this library was built from,
// baked in by the Makefile (OP_BUILD_DIGEST = sha256 of the `sha256sum` listing of DIGEST_SRCS), so a
// caller can prove the loaded binary matches its checked-out csrc/ and include/ (_lib.source_digest
// recomputes the same listing from the files), followed by ";defs=" and the build flags beyond the
// Makefile's own (empty for the product library; tools/build_variant.sh experiments name theirs).
#include <cstdint>
#include <cstring>

#include "openpose_hip.h"

#ifndef OP_BUILD_DIGEST
#error "OP_BUILD_DIGEST must be defined by the Makefile"
#endif
#ifndef OP_BUILD_FLAGS
#error "OP_BUILD_FLAGS must be defined by the Makefile"
#endif

extern "C" int op_build_info(char* out, int32_t cap) {
  static const char kInfo[] = "sha256:" OP_BUILD_DIGEST ";defs=" OP_BUILD_FLAGS;
  if (!out || cap < (int32_t)sizeof(kInfo)) return OP_ERR_INVALID;
  std::memcpy(out, kInfo, sizeof(kInfo));
  return OP_OK;
}
