// Internal C++ interface between the C ABI (capi.hip) and the kernels (codec_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kzgpot.h"

namespace kzgpot {

constexpr int kBlock = 256;  // 4 waves; one point per lane

enum class CodecOp { G1Decompress, G2Decompress, G1Transcode, G2Transcode };

// record sizes on the wire
constexpr uint64_t in_record(CodecOp op) {
  return op == CodecOp::G1Decompress ? 48 : op == CodecOp::G2Decompress ? 96 : op == CodecOp::G1Transcode ? 96 : 192;
}
constexpr uint64_t out_record(CodecOp op) {
  return (op == CodecOp::G1Decompress || op == CodecOp::G1Transcode) ? 96 : 192;
}

hipError_t launch_codec(CodecOp op, const void* d_in, void* d_out, uint64_t n, uint32_t flags,
                        unsigned long long* d_first_bad, uint8_t* d_status, hipStream_t stream);

}  // namespace kzgpot
