// CRC-32C (Castagnoli) for TFRecord framing of TensorBoard event files
// (mxtrain/obs/tensorboard.py; the reference's Mask R-CNN jobs and the Kubeflow
// Tensorboards component read tfevents).
// SSE4.2 `crc32` instruction (8 bytes per step) when the CPU has it, else slicing-by-8.
#include <cstddef>
#include <cstdint>
#include <cstring>

#define MX_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

uint32_t g_table[8][256];
bool g_init = false;

void init_tables() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    g_table[0][i] = c;
  }
  for (int t = 1; t < 8; ++t)
    for (uint32_t i = 0; i < 256; ++i)
      g_table[t][i] = (g_table[t - 1][i] >> 8) ^ g_table[0][g_table[t - 1][i] & 0xFF];
  g_init = true;
}

uint32_t crc_sw(uint32_t crc, const uint8_t* p, size_t n) {
  if (!g_init) init_tables();
  while (n >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    w ^= crc;
    crc = g_table[7][w & 0xFF] ^ g_table[6][(w >> 8) & 0xFF] ^ g_table[5][(w >> 16) & 0xFF] ^
          g_table[4][(w >> 24) & 0xFF] ^ g_table[3][(w >> 32) & 0xFF] ^
          g_table[2][(w >> 40) & 0xFF] ^ g_table[1][(w >> 48) & 0xFF] ^ g_table[0][w >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) crc = (crc >> 8) ^ g_table[0][(crc ^ *p++) & 0xFF];
  return crc;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t crc_hw(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = crc;
  while (n >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    c = __builtin_ia32_crc32di(c, w);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
  return c32;
}
#endif

}  // namespace

// crc32c of buf[0..n) (standard: init/final xor 0xFFFFFFFF applied here)
MX_EXPORT uint32_t mx_crc32c(const void* buf, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(buf);
#if defined(__x86_64__)
  if (__builtin_cpu_supports("sse4.2")) return ~crc_hw(0xFFFFFFFFu, p, n);
#endif
  return ~crc_sw(0xFFFFFFFFu, p, n);
}

// TFRecord's masked CRC: ((crc >> 15) | (crc << 17)) + 0xa282ead8
MX_EXPORT uint32_t mx_masked_crc32c(const void* buf, size_t n) {
  const uint32_t c = mx_crc32c(buf, n);
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}
