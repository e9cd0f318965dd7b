// Native drop-in for the reference's two binaries, src/bin/preprocess-kgz.rs and
// src/bin/preprocess-fastkgz.rs (their `main`s, preprocess-kgz.rs:162-199 /
// preprocess-fastkgz.rs:180-213), built as build/kzgpot-preprocess-kgz and
// build/kzgpot-preprocess-fastkgz from this one source (KZGPOT_CLI_MODE).
//
// Same files, same order of work, same messages and the same failure exit code (a Rust panic
// exits 101), minus the two things this build does not do:
//  * no download: the reference fetches the response file when ./powersoftau is missing or its
//    BLAKE2b-512 differs from POWERSOFTAU_DIGEST (preprocess-kgz.rs:32-67); here that is an error;
//  * no powersoftau_uncompressed intermediate (preprocess-kgz.rs:69-127): the GPU decodes the
//    compressed transcript straight into the arkworks file.
// Extra options (for other transcript sizes and synthetic transcripts): --transcript, --out,
// --n-log2, --gpus, --expect-digest, --no-digest-check, --output-digest, --timing. By default the work is the
// reference's: the transcript's BLAKE2b-512 is checked and the output is not hashed (the reference
// never hashes it; --output-digest adds that second stream and prints it).
#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "../../include/kzgpot.h"

#ifndef KZGPOT_CLI_MODE
#define KZGPOT_CLI_MODE KZGPOT_MODE_KZG
#endif

namespace {

// preprocess-kgz.rs:19 / preprocess-fastkgz.rs:20
const char* kPowersoftauDigest =
    "88dc1dc6914e44568e8511eace177e6ecd9da9a9bd8f67e4c0c9f215b517db4d1d54a755d051978dbb85ef947918193c93cd4cf4c99c0dc5a767d4eeb10047a4";
const char* kSectionName[] = {"tau_powers_g1", "tau_powers_g2", "alpha_tau_powers_g1", "beta_tau_powers_g1",
                              "beta_g2"};
constexpr int kPanicExit = 101;  // what a panicking Rust binary exits with

// seconds since this process started (CLOCK_BOOTTIME against /proc/self/stat's start time), for
// --timing: where a run's wall clock goes before main, in the library call, and after it
double since_start() {
  timespec now;
  clock_gettime(CLOCK_BOOTTIME, &now);
  double start = 0;
  if (FILE* f = fopen("/proc/self/stat", "r")) {
    char buf[1024];
    const size_t k = fread(buf, 1, sizeof buf - 1, f);
    fclose(f);
    buf[k] = 0;
    const char* q = strrchr(buf, ')');  // field 22 (starttime, clock ticks) counted after the comm field
    for (int field = 2; q && field < 22; field++) q = strchr(q + 1, ' ');
    if (q) start = (double)strtoull(q + 1, nullptr, 10) / (double)sysconf(_SC_CLK_TCK);
  }
  return (double)now.tv_sec + 1e-9 * (double)now.tv_nsec - start;
}

[[noreturn]] void panic_exit(const char* msg) {
  fprintf(stderr, "%s\n", msg);
  exit(kPanicExit);
}

void usage(const char* prog) {
  printf("usage: %s [--transcript PATH] [--out PATH] [--n-log2 N] [--gpus N] [--expect-digest HEX]\n"
         "          [--no-digest-check] [--output-digest]\n"
         "  --transcript PATH   powersoftau response file (default: ./powersoftau, as the reference)\n"
         "  --out PATH          output file (default: ./kzg_setup, KZG_SETUP_FILE in src/lib.rs:20)\n"
         "  --n-log2 N          2^N tau powers (default 21, TAU_POWERS_LENGTH)\n"
         "  --gpus N            GPUs to use (default 0 = every visible one)\n"
         "  --expect-digest HEX the transcript's expected BLAKE2b-512 (default: POWERSOFTAU_DIGEST)\n"
         "  --no-digest-check   skip the transcript digest check (transcripts other than the ceremony's)\n"
         "  --output-digest     also compute and print the output file's BLAKE2b-512\n"
         "  --timing            print seconds since process start at main and around the library call\n",
         prog);
}

}  // namespace

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);  // progress lines interleave with stderr as the reference's do
  const char* transcript = "powersoftau";
  const char* out = "kzg_setup";
  unsigned n_log2 = 21;
  int gpus = 0;
  bool check_digest = true, output_digest = false, timing = false;
  const char* expect = kPowersoftauDigest;
  for (int i = 1; i < argc; i++) {
    const bool has_val = i + 1 < argc;
    if (!strcmp(argv[i], "--transcript") && has_val) transcript = argv[++i];
    else if (!strcmp(argv[i], "--out") && has_val) out = argv[++i];
    else if (!strcmp(argv[i], "--n-log2") && has_val) n_log2 = (unsigned)atoi(argv[++i]);
    else if (!strcmp(argv[i], "--gpus") && has_val) gpus = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--expect-digest") && has_val) expect = argv[++i];
    else if (!strcmp(argv[i], "--no-digest-check")) check_digest = false;
    else if (!strcmp(argv[i], "--output-digest")) output_digest = true;
    else if (!strcmp(argv[i], "--timing")) timing = true;
    else if (!strcmp(argv[i], "-h") || !strcmp(argv[i], "--help")) {
      usage(argv[0]);
      return 0;
    } else {
      usage(argv[0]);
      return 2;
    }
  }
  if (n_log2 < 1 || n_log2 > 28) panic_exit("--n-log2 must be in 1..28");
  // checked up front (and normalised to the library's lowercase hex), so that a mistyped digest is
  // reported as such instead of as a failed validation after the whole transcript is hashed
  char expect_lc[129];
  if (strlen(expect) != 128) panic_exit("--expect-digest must be 128 hex characters");
  for (int i = 0; i < 128; i++) {
    if (!isxdigit((unsigned char)expect[i])) panic_exit("--expect-digest must be 128 hex characters");
    expect_lc[i] = (char)tolower((unsigned char)expect[i]);
  }
  expect_lc[128] = '\0';
  expect = expect_lc;

  // download_parameters (preprocess-kgz.rs:32-67): only the "existing file" branch exists here
  struct stat sb;
  if (stat(transcript, &sb) != 0) {
    char msg[512];
    snprintf(msg, sizeof msg,
             "called `Result::unwrap()` on an `Err` value: `%s` not found and this build has no network client "
             "(the reference downloads it here); place the response file there or pass --transcript",
             transcript);
    panic_exit(msg);
  }
  if (check_digest) printf("Checking existing %s file...\n", transcript);
  // powersoftau_uncompress size check (preprocess-kgz.rs:78-91)
  const uint64_t want = kzgpot_contribution_size(n_log2);
  if ((uint64_t)sb.st_size != want) {
    char msg[512];
    snprintf(msg, sizeof msg, "The size of `%s` should be %llu, but it's %llu, so something isn't right.", transcript,
             (unsigned long long)want, (unsigned long long)sb.st_size);
    panic_exit(msg);
  }
  const double t_main = timing ? since_start() : 0;
  if (gpus > 0) printf("Started decompressing + checking Powers of Tau on %d GPU(s)...\n", gpus);
  else printf("Started decompressing + checking Powers of Tau on every visible GPU...\n");
  char tdig[129] = {0}, odig[129] = {0};
  int bad_section = -1;
  int64_t bad_index = -1;
  const int rc = kzgpot_preprocess_ex(transcript, out, KZGPOT_CLI_MODE, n_log2, gpus, check_digest ? expect : nullptr,
                                      tdig, output_digest ? odig : nullptr, &bad_section, &bad_index);
  if (timing) printf("timing: main %.3f s after process start, library call done %.3f s after\n", t_main, since_start());
  if (rc == KZGPOT_E_DIGEST) {
    char msg[512];
    snprintf(msg, sizeof msg,
             "called `Result::unwrap()` on an `Err` value: failed validation (expected: %s, got %s); this build does "
             "not download a replacement",
             expect, tdig);
    panic_exit(msg);
  }
  if (rc > -100 && rc < 0) {  // a rejected point: the reference's unwrap() / expect() panics
    char msg[512];
    snprintf(msg, sizeof msg, "called `Result::unwrap()` on an `Err` value: point %lld of %s rejected (%s)",
             (long long)bad_index, (bad_section >= 0 && bad_section < 5) ? kSectionName[bad_section] : "?",
             kzgpot_status_name(-rc));
    panic_exit(msg);
  }
  if (rc != 0) {
    char msg[256];
    snprintf(msg, sizeof msg, "preprocess failed: %s (%d)", kzgpot_status_name(rc), rc);
    panic_exit(msg);
  }
  if (check_digest) printf("Checking passed, using existing %s file.\n", transcript);
  printf("Loaded Powers of Tau\n");
  printf("transcript BLAKE2b-512: %s\n", tdig);
  if (output_digest) printf("output BLAKE2b-512: %s\n", odig);
  printf("Done serializing. KZG parameters are stored in %s\n", out);
  // The output file is complete, closed and renamed into place; what is left is process teardown:
  // the HIP runtime's exit handlers and the library's pending buffer release. The kernel reclaims
  // all of it (device queues and memory with the /dev/kfd handle, the mappings with the address
  // space) whether or not those handlers run, so the binary leaves without them, as a Rust main
  // that returns leaves without freeing what the OS reclaims.
  fflush(stdout);
  fflush(stderr);
  _exit(0);
}
