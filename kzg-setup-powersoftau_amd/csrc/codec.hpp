// Internal C++ interface between the C ABI (capi.hip) and the kernels (codec_kernels.hip,
// g1_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kzgpot.h"

namespace kzgpot {

constexpr int kBlock = 256;  // 4 waves; one point per lane

// G1Phase1 / G2Phase1: read_g1 / read_g2 straight into the in-memory GroupAffine (load_phase1) —
// the transcode kernel in place on the input staging buffer, then the loader kernel. Host-buffer
// API only (run_host owns the staging it overwrites).
enum class CodecOp {
  G1Decompress, G2Decompress, G1Transcode, G2Transcode, G1Load, G2Load, Bn254G1Decompress, G1Phase1, G2Phase1
};

// record sizes on the wire
constexpr uint64_t in_record(CodecOp op) {
  switch (op) {
    case CodecOp::G1Decompress: return 48;
    case CodecOp::G2Decompress: return 96;
    case CodecOp::G1Transcode: return 96;
    case CodecOp::G2Transcode: return 192;
    case CodecOp::G1Load: return 96;
    case CodecOp::G2Load: return 192;
    case CodecOp::Bn254G1Decompress: return 32;
    case CodecOp::G1Phase1: return 96;
    case CodecOp::G2Phase1: return 192;
  }
  return 0;
}
constexpr uint64_t out_record(CodecOp op) {
  switch (op) {
    case CodecOp::G1Decompress: return 96;
    case CodecOp::G2Decompress: return 192;
    case CodecOp::G1Transcode: return 96;
    case CodecOp::G2Transcode: return 192;
    case CodecOp::G1Load: return KZGPOT_G1_ARK_MONT_BYTES;
    case CodecOp::G2Load: return KZGPOT_G2_ARK_MONT_BYTES;
    case CodecOp::Bn254G1Decompress: return 64;
    case CodecOp::G1Phase1: return KZGPOT_G1_ARK_MONT_BYTES;
    case CodecOp::G2Phase1: return KZGPOT_G2_ARK_MONT_BYTES;
  }
  return 0;
}

// phase 1 marks a rejected point's record with this value in x's top word (phase 2 then skips it)
constexpr uint32_t kPoison = 0xffffffffu;

// where phase 2 (k_g1_check / k_g2_check) reads its record (codec_kernels.hip "phase 2")
enum class Src { ArkInPlace, PairingBE, PairingBEInPlace };
constexpr bool src_in_place(Src s) { return s != Src::PairingBE; }

// G1 kernels (g1_kernels.hip, its own translation unit: compiled with the iterative ILP scheduler):
// G1Decompress (fused or split), G1Transcode, and G1Phase1's in-place transcode (in = nullptr)
hipError_t launch_g1(CodecOp op, const uint4* in, uint4* out, uint64_t n, uint32_t flags,
                     unsigned long long* d_first_bad, uint8_t* d_status, hipStream_t stream);

// loader kernels (load_kernels.hip)
hipError_t launch_load(bool g2, const void* d_in, void* d_out, uint64_t n, unsigned long long* d_first_bad,
                       uint8_t* d_status, hipStream_t stream);

// BN254 G1 codec (bn254_kernels.hip)
hipError_t launch_bn254(const void* d_in, void* d_out, uint64_t n, unsigned long long* d_first_bad,
                        uint8_t* d_status, hipStream_t stream);

hipError_t launch_codec(CodecOp op, const void* d_in, void* d_out, uint64_t n, uint32_t flags,
                        unsigned long long* d_first_bad, uint8_t* d_status, hipStream_t stream);

}  // namespace kzgpot
