/* CPU ORACLE (test infrastructure only): RFC 7693 BLAKE2b-512, see blake2b_ref.c. */
#pragma once
#include <stddef.h>
#include <stdint.h>

typedef struct {
  uint64_t h[8], t[2];
  uint8_t buf[128];
  size_t fill;
} oracle_blake2b_state;

void oracle_blake2b_init(oracle_blake2b_state* s);
void oracle_blake2b_update(oracle_blake2b_state* s, const uint8_t* p, size_t n);
void oracle_blake2b_final(oracle_blake2b_state* s, uint8_t out[64]);
int oracle_blake2b(const uint8_t* p, size_t n, uint8_t out[64]);
