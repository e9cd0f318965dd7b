// BLAKE2b-512 (RFC 7693), streaming. See blake2b.cpp.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace kzgpot {

class Blake2b {
 public:
  Blake2b() { init(); }
  void init();
  void update(const uint8_t* p, size_t len);
  void finalize(uint8_t out[64]);

 private:
  void compress(const uint8_t* block, bool last);
  uint64_t h_[8];
  unsigned __int128 t_;
  uint8_t buf_[128];
  size_t n_;
};

void blake2b_512(const uint8_t* data, size_t len, uint8_t out[64]);
void to_hex(const uint8_t d[64], char hex[129]);

}  // namespace kzgpot
