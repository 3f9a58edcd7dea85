// The library's own CPU route (host_crc.cpp): per-call digests of small host buffers, and every
// host-buffer call when no HIP device is visible. It plays the role the reference's class-init
// provider chain gives its JNI SSE4.2 path (circe-checksum/src/main/java/com/scurrilous/circe/
// checksum/Crc32cIntChecksum.java:28-36): a call never fails for lack of a device. Batch entry
// points never take this route.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace bkd {
namespace host {

// Raw register update: reg' = (reg * x^(8n) + M(x) * x^32) mod P (reflected, no complements).
// resume(prev, M) = ~crc_raw(algo, ~prev, M).
uint32_t crc_raw(int algo, uint32_t reg, const uint8_t* p, size_t n);

// Whether crc_raw has the AVX-512 VPCLMULQDQ path on this CPU (it then beats a GPU round trip
// for single host buffers up to tens of MiB).
bool has_wide_fold();

// Which implementation crc_raw dispatches to on this CPU: "vpclmul512+pclmul+sse4.2", "pclmul+sse4.2",
// "pclmul", "slice8".
const char* impl_name();

}  // namespace host
}  // namespace bkd
