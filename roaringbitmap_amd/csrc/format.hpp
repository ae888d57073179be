// format.hpp — host-side RoaringFormatSpec codec and canonical-form validation.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace rbg {

// Host SoA batch; payload offsets are 16-byte aligned, Bitmap payloads 8192-aligned when
// produced by layout_for_device().
struct HostSoA {
  uint32_t nb = 0;
  std::vector<uint64_t> begin{0};
  std::vector<uint16_t> key;
  std::vector<uint8_t> type;
  std::vector<uint32_t> card;
  std::vector<uint16_t> nruns;
  std::vector<uint64_t> off;
  std::vector<uint8_t> payload;
  uint64_t nc() const { return key.size(); }
};

// Parse one serialized bitmap (RoaringArray.deserialize, RoaringArray.java:276-348 / 547-629)
// and append it to `out`.  Returns 0, RB_EFORMAT (cookie / size / truncation) or RB_EINVAL
// (non-canonical content).
int parse_serialized(const uint8_t *buf, uint64_t len, HostSoA &out, std::string &err);

// Check one container of a host SoA for the canonical form the engine relies on.
int validate_container(uint16_t type, uint32_t card, uint32_t nruns, const uint8_t *payload, std::string &err);

// RoaringArray.serializedSizeInBytes / serialize (RoaringArray.java:851-953) for bitmap b.
uint64_t serialized_size(const HostSoA &s, uint32_t b);
void serialize_bitmap(const HostSoA &s, uint32_t b, uint8_t *dst);

} // namespace rbg
