// CRC-32 of PNG chunks (zlib's crc32 value, PCLMULQDQ folding when available).
#pragma once

#include <cstddef>
#include <cstdint>

namespace zpx {
uint32_t crc32_fast(uint32_t crc, const uint8_t *buf, size_t len);
}
