/*
 * kzgpot — MI355X-native Powers-of-Tau → arkworks KZG preprocessor: the C ABI.
 *
 * Drop-in boundary for the per-point hot path of heliaxdev/kzg-setup-powersoftau. The reference
 * is a Rust crate with no FFI; each entry point below names the reference code it replaces
 * (paths relative to the reference repo root). A Rust crate binds these with `extern "C"` (see
 * INTEGRATION.md); the Python package and the tests bind them with ctypes.
 *
 * Conventions
 *  - Plain pointers and sizes only. Host variants take host buffers and are synchronous. `_dev`
 *    variants take device pointers (HBM) and a hipStream_t passed as void*; they are
 *    asynchronous and report errors through a device-side key (see kzgpot_decode_bad_key).
 *  - Point formats: G1 compressed 48 B / uncompressed 96 B, G2 compressed 96 B / uncompressed
 *    192 B. "pairing" = zcash pairing 0.14.2 big-endian encodings as written by powersoftau;
 *    "ark" = ark-serialize 0.2 `serialize_uncompressed` (little-endian, SWFlags in the top byte).
 *  - Return value: 0 = every point accepted; -(status) of the FIRST rejected point (smallest
 *    index, deterministic) when a point is rejected; <= KZGPOT_E_INVALID_ARG on API/runtime errors.
 *    Rejected points' output records are zero-filled. The reference panics on the first bad point
 *    (`unwrap`, preprocess-kgz.rs:110,142); callers that want that behaviour abort on != 0.
 *  - Accept/reject and output bytes are bit-exact with the reference for every input; the error
 *    CLASS is informative (the reference's own class depends on which stage trips first).
 */
#ifndef KZGPOT_H
#define KZGPOT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- per-point status / errors */
#define KZGPOT_OK 0
#define KZGPOT_ST_COMPRESSION_MODE 1 /* pairing GroupDecodingError::UnexpectedCompressionMode */
#define KZGPOT_ST_UNEXPECTED_INFO 2  /* pairing GroupDecodingError::UnexpectedInformation */
#define KZGPOT_ST_NOT_IN_FIELD 3     /* pairing CoordinateDecodingError / ark InvalidData (coord >= p) */
#define KZGPOT_ST_NOT_ON_CURVE 4     /* pairing GroupDecodingError::NotOnCurve (x^3+b non-residue) */
#define KZGPOT_ST_NOT_IN_SUBGROUP 5  /* ark InvalidData from is_in_correct_subgroup_assuming_on_curve */
#define KZGPOT_ST_UNEXPECTED_FLAGS 6 /* ark SerializationError::UnexpectedFlags */
#define KZGPOT_ST_INFINITY 7         /* point at infinity reaching read_g1/read_g2: the reference panics */

#define KZGPOT_E_INVALID_ARG (-100)
#define KZGPOT_E_DEVICE (-101)  /* HIP runtime failure or no usable GPU: the product path never falls back to CPU */
#define KZGPOT_E_IO (-102)
#define KZGPOT_E_SIZE (-103)    /* transcript size != powersoftau CONTRIBUTION_BYTE_SIZE (preprocess-kgz.rs:83-91) */
#define KZGPOT_E_DIGEST (-104)  /* BLAKE2b-512 mismatch (preprocess-kgz.rs:51-61, src/lib.rs:147-157) */
#define KZGPOT_E_NETWORK (-105) /* download requested: this build has no network client */
#define KZGPOT_E_RANK_FAILED (-106) /* multi-GPU: a rank (maybe this one) could not decode its share */
#define KZGPOT_E_TIMEOUT (-107)     /* multi-GPU: kzgpot_comm_wait gave up; the communicator is aborted */
/* Host resources ran out: host memory (std::bad_alloc), the file path's 0.6-1.6 GB buffer mappings,
 * or a host thread (EAGAIN under a process or thread limit). The call has joined every thread it
 * started and removed its temporary output file; nothing crossed the C ABI as an exception. The
 * reference returns a Result here (Accumulator::deserialize, preprocess-kgz.rs:105-110). */
#define KZGPOT_E_OUT_OF_MEMORY (-108)

/* ---------------------------------------------------------------- flags */
/* Decompression only (powersoftau CheckForCorrectness::No with no read_g1 afterwards — the βτG1 /
 * βG2 sections in preprocess-kgz). The point at infinity is then legal and is emitted as ark
 * GroupAffine::zero(). Default (flag clear): the full reference chain of a point that is read
 * back by read_g1/read_g2 — infinity rejected, subgroup checked. */
#define KZGPOT_NO_SUBGROUP_CHECK 0x1u
/* Use the reference's own subgroup algorithm (ark mul_bits by r, 255-bit double-and-add) instead
 * of the endomorphism test. Same boolean for every point; ~3x slower. For cross-validation. */
#define KZGPOT_SUBGROUP_REF 0x2u
/* Checked G1 / G2 decompression as two launches (decompress, then the arkworks check in place on
 * its output — the split kernels) instead of the fused one-pass kernel. Same output and statuses;
 * for A/B measurement. */
#define KZGPOT_SPLIT_PHASES 0x4u

/* ---------------------------------------------------------------- hot path, host buffers */
/* Compressed G1 (48 B each, pairing) → ark uncompressed (96 B each).
 * Replaces, per point: pairing G1Compressed::into_affine_unchecked (via powersoftau
 * Accumulator::deserialize, src/bin/preprocess-kgz.rs:105-110) → G1Uncompressed (preprocess-kgz.rs:122)
 * → read_g1 (src/lib.rs:41-54, incl. ark subgroup check) → serialize_uncompressed (preprocess-kgz.rs:188-194). */
int kzgpot_g1_decompress(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags, int64_t* first_bad);
/* Compressed G2 (96 B) → ark uncompressed (192 B). Same chain with read_g2 (src/lib.rs:56-80) and the
 * fastkgz G2 emit (src/bin/preprocess-fastkgz.rs:206-208). */
int kzgpot_g2_decompress(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags, int64_t* first_bad);
/* Pairing-uncompressed G1 (96 B) → ark (96 B): the read_g1 loop alone (src/lib.rs:41-54;
 * preprocess-kgz.rs:140-153; load_phase1 src/lib.rs:92-110). flags: KZGPOT_SUBGROUP_REF only. */
int kzgpot_g1_transcode_uncompressed(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags, int64_t* first_bad);
/* Pairing-uncompressed G2 (192 B) → ark (192 B): the read_g2 loop (src/lib.rs:56-80). */
int kzgpot_g2_transcode_uncompressed(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags, int64_t* first_bad);

/* As above, also writing one status byte per point (KZGPOT_ST_*) into status[n] (may be NULL). */
int kzgpot_g1_decompress_ex(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags, int64_t* first_bad, uint8_t* status);
int kzgpot_g2_decompress_ex(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags, int64_t* first_bad, uint8_t* status);
int kzgpot_g1_transcode_uncompressed_ex(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags, int64_t* first_bad, uint8_t* status);
int kzgpot_g2_transcode_uncompressed_ex(const uint8_t* in, size_t n, uint8_t* out, uint32_t flags, int64_t* first_bad, uint8_t* status);

/* ---------------------------------------------------------------- hot path, device buffers (async) */
/* d_bad_key: one device uint64 that the call resets to UINT64_MAX (on `stream`) and that the
 * kernel lowers with atomicMin((index << 8) | status). d_status may be NULL. */
int kzgpot_g1_decompress_dev(const void* d_in, size_t n, void* d_out, uint32_t flags, uint64_t* d_bad_key,
                             uint8_t* d_status, void* stream);
int kzgpot_g2_decompress_dev(const void* d_in, size_t n, void* d_out, uint32_t flags, uint64_t* d_bad_key,
                             uint8_t* d_status, void* stream);
int kzgpot_g1_transcode_uncompressed_dev(const void* d_in, size_t n, void* d_out, uint32_t flags,
                                         uint64_t* d_bad_key, uint8_t* d_status, void* stream);
int kzgpot_g2_transcode_uncompressed_dev(const void* d_in, size_t n, void* d_out, uint32_t flags,
                                         uint64_t* d_bad_key, uint8_t* d_status, void* stream);
/* Host-side decode of a bad key copied back from the device: returns 0 (none) or -(status) and
 * sets *first_bad to the index (or -1). The multi-rank key KZGPOT_KEY_RANK_FAILED (0) decodes to
 * KZGPOT_E_RANK_FAILED with *first_bad = -1: a gathered buffer with a failed peer is never "ok". */
int kzgpot_decode_bad_key(uint64_t key, int64_t* first_bad);

/* ---------------------------------------------------------------- file pipeline (next-row §8f) */
#define KZGPOT_MODE_KZG 0     /* src/bin/preprocess-kgz.rs: Powers + VerifierKey file */
#define KZGPOT_MODE_FASTKZG 1 /* src/bin/preprocess-fastkgz.rs: UniversalParams + powers_of_h file */
/* powersoftau CONTRIBUTION_BYTE_SIZE for 2^n_log2 powers (603,981,040 at n_log2 = 21). */
uint64_t kzgpot_contribution_size(uint32_t n_log2);
/* Output size of `mode` for 2^n_log2 powers (kgz 603,980,256 / fastkzg 1,006,633,248 at 21). */
uint64_t kzgpot_output_size(uint32_t n_log2, int mode);
/* preprocess-{kgz,fastkgz} main (preprocess-kgz.rs:162-199, preprocess-fastkgz.rs:180-213) minus the
 * download: reads the response transcript at `transcript_path`, checks its size, decompresses and
 * checks every section, writes `out_path`. No intermediate file.
 * n_gpus is a SHARD count (0 = one per visible GPU; at most 64): each section is split into n_gpus contiguous
 * shards, each driven by a host thread on GPU (current + k) mod device_count — more shards than
 * GPUs put several shards on one GPU. The caller's current device is restored on return.
 * File path: the transcript is pread() in 32 MiB pieces while the GPU decodes what has arrived;
 * the output is pwrite()n as it lands into a temporary file "<out_path>.kzgpot-tmp-XXXXXX"
 * (mkstemp: unique per call) in the same directory, renamed over out_path only on success and
 * removed on any error, so out_path is either the complete file or untouched.
 * Returns 0 or a negative error; on a rejected point *bad_section (0 τG1, 1 τG2, 2 ατG1, 3 βτG1,
 * 4 βG2) and *bad_index locate it (pointers may be NULL). */
int kzgpot_preprocess(const char* transcript_path, const char* out_path, int mode, uint32_t n_log2, int n_gpus,
                      int* bad_section, int64_t* bad_index);
/* Same, on in-memory buffers (out must hold kzgpot_output_size bytes). */
int kzgpot_preprocess_buffer(const uint8_t* transcript, size_t len, uint8_t* out, int mode, uint32_t n_log2,
                             int n_gpus, int* bad_section, int64_t* bad_index);
/* With the BLAKE2b-512 digests (src/lib.rs:129; the reference checks the transcript against
 * POWERSOFTAU_DIGEST, preprocess-kgz.rs:19,51-61, and publishes the outputs' digests,
 * src/lib.rs:21-22). Hashing runs on host threads beside the GPU pass: the transcript from the
 * start, the output section by section as the GPU finishes it. expect_transcript_digest (128 hex
 * chars, may be NULL): a mismatch returns KZGPOT_E_DIGEST (and no output file is written).
 * transcript_digest / output_digest (may be NULL): receive 128 hex chars + NUL. */
int kzgpot_preprocess_ex(const char* transcript_path, const char* out_path, int mode, uint32_t n_log2, int n_gpus,
                         const char* expect_transcript_digest, char* transcript_digest, char* output_digest,
                         int* bad_section, int64_t* bad_index);
int kzgpot_preprocess_buffer_ex(const uint8_t* transcript, size_t len, uint8_t* out, int mode, uint32_t n_log2,
                                int n_gpus, const char* expect_transcript_digest, char* transcript_digest,
                                char* output_digest, int* bad_section, int64_t* bad_index);
/* BLAKE2b-512 (unkeyed, 64-byte digest) of a host buffer — blake2b_simd::State::new() (src/lib.rs:129). */
int kzgpot_blake2b(const uint8_t* data, size_t len, uint8_t* digest64);

/* ---------------------------------------------------------------- loader mirror (next-row §8f 2) */
/* ark-ec 0.2 GroupAffine in memory (what `deserialize_unchecked` returns): each Fp as 6 LE u64 in
 * ark-ff Montgomery form (R = 2^384), then `infinity` (u8) and zero padding to 8 B:
 *   G1 104 B = x[48] y[48] inf[1] pad[7];  G2 200 B = x.c0 x.c1 y.c0 y.c1 [4 x 48] inf[1] pad[7].
 * A Rust caller reads these as #[repr(C)] mirrors of GroupAffine. */
#define KZGPOT_G1_ARK_MONT_BYTES 104
#define KZGPOT_G2_ARK_MONT_BYTES 200
/* ark-uncompressed G1 (96 B) → GroupAffine (104 B): ArkG1Affine::deserialize_unchecked (src/lib.rs:180,
 * 183) — coordinates < p and SWFlags checked, NO curve and NO subgroup check. */
int kzgpot_g1_deserialize_unchecked(const uint8_t* in, size_t n, uint8_t* out, int64_t* first_bad);
/* ark-uncompressed G2 (192 B) → GroupAffine (200 B): ArkG2Affine::deserialize_unchecked (src/lib.rs:209-215). */
int kzgpot_g2_deserialize_unchecked(const uint8_t* in, size_t n, uint8_t* out, int64_t* first_bad);
int kzgpot_g1_deserialize_unchecked_ex(const uint8_t* in, size_t n, uint8_t* out, int64_t* first_bad, uint8_t* status);
int kzgpot_g2_deserialize_unchecked_ex(const uint8_t* in, size_t n, uint8_t* out, int64_t* first_bad, uint8_t* status);
int kzgpot_g1_deserialize_unchecked_dev(const void* d_in, size_t n, void* d_out, uint64_t* d_bad_key,
                                        uint8_t* d_status, void* stream);
int kzgpot_g2_deserialize_unchecked_dev(const void* d_in, size_t n, void* d_out, uint64_t* d_bad_key,
                                        uint8_t* d_status, void* stream);
/* load_kzg_setup (src/lib.rs:174-195) for 2^n_log2 powers (the reference fixes n_log2 = 21):
 * powers_of_g (2N-1 G1), powers_of_gamma_g (N G1), vk = g, gamma_g (G1), h, beta_h (G2) =
 * 2 x 104 + 2 x 200 B (VerifierKey::deserialize_unchecked; prepared_h / prepared_beta_h are the
 * caller's `h.into()` / `beta_h.into()`). Output buffers in the layout above. Trailing bytes are
 * ignored, as by the reference's sequential reader; a short file is KZGPOT_E_SIZE. On a rejected
 * point *bad_section (0 powers_of_g, 1 powers_of_gamma_g, 2 vk/h-beta_h, 3 powers_of_h) and
 * *bad_index locate it. */
int kzgpot_load_kzg_setup(const char* path, uint32_t n_log2, uint8_t* powers_of_g, uint8_t* powers_of_gamma_g,
                          uint8_t* vk, int* bad_section, int64_t* bad_index);
int kzgpot_load_kzg_setup_buffer(const uint8_t* file, size_t len, uint32_t n_log2, uint8_t* powers_of_g,
                                 uint8_t* powers_of_gamma_g, uint8_t* vk, int* bad_section, int64_t* bad_index);
/* load_fastkzg_setup (src/lib.rs:197-228): powers_of_g, powers_of_gamma_g, h_beta_h = h, beta_h
 * (2 x 200 B, as read: prepared_beta_h = beta_h.into()), powers_of_h (N G2). UniversalParams.beta_h
 * is powers_of_h[1] in the reference (src/lib.rs:221), not the beta_h read from the file. NB: the
 * reference opens KZG_SETUP_FILE here (src/lib.rs:198); this entry point takes the path. */
int kzgpot_load_fastkzg_setup(const char* path, uint32_t n_log2, uint8_t* powers_of_g, uint8_t* powers_of_gamma_g,
                              uint8_t* h_beta_h, uint8_t* powers_of_h, int* bad_section, int64_t* bad_index);
int kzgpot_load_fastkzg_setup_buffer(const uint8_t* file, size_t len, uint32_t n_log2, uint8_t* powers_of_g,
                                     uint8_t* powers_of_gamma_g, uint8_t* h_beta_h, uint8_t* powers_of_h,
                                     int* bad_section, int64_t* bad_index);

/* load_phase1(exp) (src/lib.rs:82-121, Phase1Parameters src/lib.rs:30-39), next-row §8f 3: a
 * phase1radix2m{exp} file = alpha, beta_g1 (G1), beta_g2 (G2), then coeffs_g1, coeffs_g2,
 * alpha_coeffs_g1, beta_coeffs_g1 (2^exp points each), every point read by read_g1 / read_g2
 * (src/lib.rs:41-80: pairing uncompressed, byte reorder, ark deserialize_uncompressed with the
 * subgroup check) into the in-memory GroupAffine layout (104 / 200 B per point). The reference
 * hardcodes the path "../phase1radix2m{exp}" (src/lib.rs:84); here it is an argument. Trailing
 * bytes are ignored; a short file is KZGPOT_E_SIZE. *bad_section: 0 alpha, 1 beta_g1, 2 beta_g2,
 * 3 coeffs_g1, 4 coeffs_g2, 5 alpha_coeffs_g1, 6 beta_coeffs_g1. */
uint64_t kzgpot_phase1_size(uint32_t exp);
int kzgpot_load_phase1(const char* path, uint32_t exp, uint8_t* alpha, uint8_t* beta_g1, uint8_t* beta_g2,
                       uint8_t* coeffs_g1, uint8_t* coeffs_g2, uint8_t* alpha_coeffs_g1, uint8_t* beta_coeffs_g1,
                       int* bad_section, int64_t* bad_index);
int kzgpot_load_phase1_buffer(const uint8_t* file, size_t len, uint32_t exp, uint8_t* alpha, uint8_t* beta_g1,
                              uint8_t* beta_g2, uint8_t* coeffs_g1, uint8_t* coeffs_g2, uint8_t* alpha_coeffs_g1,
                              uint8_t* beta_coeffs_g1, int* bad_section, int64_t* bad_index);

/* ---------------------------------------------------------------- BN254 (config 5, next-row §8f 4) */
/* No reference counterpart: the same path instantiated for ark-bn254 0.2 G1 (cofactor 1).
 * ark compressed (32 B: x LE, SWFlags bit7 PositiveY / bit6 Infinity in byte 31) → ark
 * uncompressed (64 B) = ark-ec 0.2 GroupAffine::deserialize + serialize_uncompressed. The point
 * at infinity is legal (→ ark zero()). Statuses: 3 NotInField, 4 NotOnCurve, 6 UnexpectedFlags. */
int kzgpot_bn254_g1_decompress(const uint8_t* in, size_t n, uint8_t* out, int64_t* first_bad);
int kzgpot_bn254_g1_decompress_ex(const uint8_t* in, size_t n, uint8_t* out, int64_t* first_bad, uint8_t* status);
int kzgpot_bn254_g1_decompress_dev(const void* d_in, size_t n, void* d_out, uint64_t* d_bad_key, uint8_t* d_status,
                                   void* stream);

/* ---------------------------------------------------------------- multi-GPU, RCCL inside */
/* north_star: "the τ^i array shards trivially across the 8 GPUs of one node with a final RCCL
 * all-gather over xGMI to produce one contiguous arkworks buffer". Replaces the reference's only
 * parallel stage, the chunked decompression of powersoftau's Accumulator::deserialize
 * (src/bin/preprocess-kgz.rs:105-110), whose workers fill disjoint slices of one Vec — here the
 * slices live on different GPUs and RCCL assembles them. One process (or thread) per GPU.
 *   rank 0: kzgpot_comm_unique_id(id); ship the 128 bytes to every rank (MPI, torch.distributed,
 *   a file, ...); every rank, with its GPU current: kzgpot_comm_init(&comm, id, nranks, rank).
 * RCCL is bound at first use with dlopen("librccl.so.1") (in a torch process: the RCCL torch has
 * already loaded). */
#define KZGPOT_COMM_ID_BYTES 128
int kzgpot_comm_unique_id(uint8_t* id);
int kzgpot_comm_init(void** comm, const uint8_t* id, int nranks, int rank); /* collective */
int kzgpot_comm_destroy(void* comm);
#define KZGPOT_OP_G1_DECOMPRESS 0
#define KZGPOT_OP_G2_DECOMPRESS 1
#define KZGPOT_OP_G1_TRANSCODE 2
#define KZGPOT_OP_G2_TRANSCODE 3
#define KZGPOT_OP_BN254_G1_DECOMPRESS 4
/* Block-cyclic layout of n points over nranks x chunks: *block = floor(n / (nranks chunks)) points
 * per block, *tail = the n - nranks chunks block points at the end. Rank k owns blocks
 * c nranks + k (global points [(c nranks + k) block, +block)), c = 0..chunks-1; every rank also
 * decodes the tail. */
int kzgpot_shard_layout(uint64_t n, int nranks, uint32_t chunks, uint64_t* block, uint64_t* tail);
/* Collective, asynchronous on `stream` (a hipStream_t of the communicator's GPU). d_in_local =
 * this rank's input records: its `chunks` owned blocks in chunk order, then the tail (chunks x
 * block + tail records). d_out = all n output records (HBM, every rank). Each chunk is decoded
 * on `stream` and then all-gathered in place (ncclAllGather on the communicator's own stream)
 * while the next chunk decodes. *d_bad_key = the first rejected point over ALL ranks as
 * (global index << 8) | status, or all ones (decode with kzgpot_decode_bad_key); rejected
 * records are zero-filled as in the single-GPU calls. `stream` waits for the gathers.
 * Collective contract: every rank calls with the same op, n, chunks and flags (the layout is
 * derived from them). Errors never desynchronise the ranks:
 *  - argument errors (identical on every rank, since the arguments are) return
 *    KZGPOT_E_INVALID_ARG before any collective is queued;
 *  - a local HIP failure (a decode launch, an event, the key buffer) stops this rank's decoding
 *    but every collective is still issued, so no peer waits forever; the all-reduced key is then
 *    KZGPOT_KEY_RANK_FAILED on every rank (kzgpot_comm_wait returns KZGPOT_E_RANK_FAILED) and
 *    this call returns KZGPOT_E_DEVICE. The communicator stays usable;
 *  - a failing RCCL call aborts the communicator (ncclCommAbort; later calls return
 *    KZGPOT_E_DEVICE) and returns KZGPOT_E_DEVICE. Peers then fail in their own RCCL calls or
 *    time out in kzgpot_comm_wait.
 * Calls on one communicator are ordered: each waits (on its `stream`) for the previous call's
 * collectives before touching the communicator's key buffers, whatever stream that call used. */
int kzgpot_decode_allgather_dev(void* comm, int op, const void* d_in_local, uint64_t n, uint32_t chunks, void* d_out,
                                uint32_t flags, uint64_t* d_bad_key, void* stream);
#define KZGPOT_KEY_RANK_FAILED 0ull /* the all-reduced key when some rank failed (no real key is 0: status >= 1) */
/* Host-side completion of kzgpot_decode_allgather_dev: waits for `stream` (polling, so that a
 * stuck collective cannot hang the caller), then decodes *d_bad_key. Returns 0 (every point
 * accepted), -(status) of the first rejected point (*first_bad = its global index),
 * KZGPOT_E_RANK_FAILED when a rank could not decode its share, KZGPOT_E_DEVICE on a device or
 * RCCL asynchronous error, or KZGPOT_E_TIMEOUT after timeout_ms (0 = no limit) — the last two
 * abort the communicator, which makes RCCL's kernels on this rank exit (the CUDA-style watchdog
 * a torch process group runs). first_bad may be NULL. */
int kzgpot_comm_wait(void* comm, const uint64_t* d_bad_key, int64_t* first_bad, uint32_t timeout_ms, void* stream);
/* What RCCL itself reports for the communicator (ncclCommCount / ncclCommUserRank /
 * ncclCommCuDevice): the rank count, this rank and its HIP device. Any pointer may be NULL.
 * KZGPOT_E_DEVICE once the communicator is aborted. bench.py puts these in its line, so an N-GPU
 * number carries RCCL's own proof of N. */
int kzgpot_comm_size(void* comm, int* nranks, int* rank, int* device);
/* Failure injection (kzgpot_comm_inject_fault, kzgpot_test_inject_host_fault) and the
 * KZGPOT_RCCL_LIB override exist only in the test build libkzgpot_test.so (tests/kzgpot_test_hooks.h); this library binds librccl.so.1. */

/* ---------------------------------------------------------------- misc */
const char* kzgpot_status_name(int status);  /* name of a KZGPOT_ST_* or KZGPOT_E_* code */
int kzgpot_device_count(void);               /* visible HIP devices (0 if none) */
const char* kzgpot_version(void);

#ifdef __cplusplus
}
#endif
#endif /* KZGPOT_H */
