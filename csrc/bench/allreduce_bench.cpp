// allreduce_bench.cpp - RCCL all-reduce bandwidth against message (bucket)
// size on the GPUs of one node, one communicator per GPU driven from one
// process (ncclCommInitAll + group calls).  Picks the gradient bucket size of
// the data-parallel path (root.common.engine.dp.bucket_mb, docs/PARALLEL.md)
// from measurement instead of by analogy with NVLink numbers: on MI355X the
// GPUs are joined point-to-point by xGMI (7 links per GPU), so a ring is
// bound per link and small buckets fall into the latency regime.
//
// "a C++ all-reduce micro-benchmark (RCCL ncclAllReduce on
// device buffers) establishes the per-bucket latency/bandwidth curve".
// Replaces nothing in the reference (it has no collectives; its master
// aggregated gradients on the host, veles/server.py:369-414).
//
//   allreduce_bench [ngpus] [min_mb] [max_mb] [iters] [dtype f32|bf16]
//
// Prints one line per size: bytes, time per all-reduce (mean over iters,
// after warmup), algbw = bytes / t and busbw = algbw * 2 (n - 1) / n (the
// per-link rate of a ring, comparable across GPU counts), and a JSON line at
// the end.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define HIPCHECK(x)                                                        \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,       \
                   hipGetErrorString(e_));                                 \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)
#define NCCLCHECK(x)                                                       \
  do {                                                                     \
    ncclResult_t r_ = (x);                                                 \
    if (r_ != ncclSuccess) {                                               \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,       \
                   ncclGetErrorString(r_));                                \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

int main(int argc, char** argv) {
  int avail = 0;
  HIPCHECK(hipGetDeviceCount(&avail));
  const int n = argc > 1 ? std::atoi(argv[1]) : avail;
  const double min_mb = argc > 2 ? std::atof(argv[2]) : 1.0;
  const double max_mb = argc > 3 ? std::atof(argv[3]) : 256.0;
  const int iters = argc > 4 ? std::atoi(argv[4]) : 20;
  const bool bf16 = argc > 5 && std::strcmp(argv[5], "bf16") == 0;
  if (n < 1 || n > avail) {
    std::fprintf(stderr, "need 1..%d GPUs, asked %d\n", avail, n);
    return 2;
  }
  const ncclDataType_t dt = bf16 ? ncclBfloat16 : ncclFloat32;
  const size_t esz = bf16 ? 2 : 4;
  const size_t max_bytes = (size_t)(max_mb * 1048576.0);

  std::vector<int> devs(n);
  for (int i = 0; i < n; ++i) devs[i] = i;
  std::vector<ncclComm_t> comms(n);
  NCCLCHECK(ncclCommInitAll(comms.data(), n, devs.data()));
  std::vector<hipStream_t> streams(n);
  // out-of-place (send != recv), as the trainer's bucket reduce is not: with
  // one GPU RCCL then still moves the bytes (a device copy) instead of
  // returning at once, so the 1-GPU line is the copy floor
  std::vector<void*> buf(n), rbuf(n);
  std::vector<hipEvent_t> e0(n), e1(n);
  for (int i = 0; i < n; ++i) {
    HIPCHECK(hipSetDevice(i));
    HIPCHECK(hipStreamCreateWithFlags(&streams[i], hipStreamNonBlocking));
    HIPCHECK(hipMalloc(&buf[i], max_bytes));
    HIPCHECK(hipMalloc(&rbuf[i], max_bytes));
    HIPCHECK(hipMemset(buf[i], 0, max_bytes));
    HIPCHECK(hipEventCreate(&e0[i]));
    HIPCHECK(hipEventCreate(&e1[i]));
  }
  int rv = 0;
  NCCLCHECK(ncclGetVersion(&rv));
  std::printf("# RCCL %d, %d GPU(s), dtype %s, %d iterations per size\n", rv,
              n, bf16 ? "bf16" : "f32", iters);
  std::printf("%12s %12s %12s %12s\n", "bytes", "us", "algbw GB/s",
              "busbw GB/s");

  auto run = [&](size_t count) {
    NCCLCHECK(ncclGroupStart());
    for (int i = 0; i < n; ++i)
      NCCLCHECK(ncclAllReduce(buf[i], rbuf[i], count, dt, ncclSum, comms[i],
                              streams[i]));
    NCCLCHECK(ncclGroupEnd());
  };
  std::string json = "{\"tool\": \"allreduce_bench\", \"gpus\": " +
                     std::to_string(n) + ", \"dtype\": \"" +
                     (bf16 ? "bf16" : "f32") + "\", \"rccl\": " +
                     std::to_string(rv) + ", \"sizes\": [";
  bool firstj = true;
  for (double mb = min_mb; mb <= max_mb * 1.0001; mb *= 2.0) {
    const size_t bytes = (size_t)(mb * 1048576.0) / esz * esz;
    const size_t count = bytes / esz;
    for (int w = 0; w < 3; ++w) run(count);  // warmup
    for (int i = 0; i < n; ++i) {
      HIPCHECK(hipSetDevice(i));
      HIPCHECK(hipStreamSynchronize(streams[i]));
      HIPCHECK(hipEventRecord(e0[i], streams[i]));
    }
    for (int it = 0; it < iters; ++it) run(count);
    float worst = 0.f;
    for (int i = 0; i < n; ++i) {
      HIPCHECK(hipSetDevice(i));
      HIPCHECK(hipEventRecord(e1[i], streams[i]));
      HIPCHECK(hipEventSynchronize(e1[i]));
      float ms = 0.f;
      HIPCHECK(hipEventElapsedTime(&ms, e0[i], e1[i]));
      if (ms > worst) worst = ms;
    }
    const double us = 1e3 * worst / iters;
    const double alg = (double)bytes / (us * 1e-6) / 1e9;
    const double bus = n > 1 ? alg * 2.0 * (n - 1) / n : alg;
    std::printf("%12zu %12.1f %12.1f %12.1f\n", bytes, us, alg, bus);
    char item[160];
    std::snprintf(item, sizeof(item),
                  "%s{\"bytes\": %zu, \"us\": %.1f, \"algbw\": %.1f, "
                  "\"busbw\": %.1f}",
                  firstj ? "" : ", ", bytes, us, alg, bus);
    json += item;
    firstj = false;
  }
  json += "]}";
  std::printf("%s\n", json.c_str());
  for (int i = 0; i < n; ++i) {
    HIPCHECK(hipSetDevice(i));
    HIPCHECK(hipFree(buf[i]));
    HIPCHECK(hipFree(rbuf[i]));
    HIPCHECK(hipStreamDestroy(streams[i]));
    HIPCHECK(hipEventDestroy(e0[i]));
    HIPCHECK(hipEventDestroy(e1[i]));
    ncclCommDestroy(comms[i]);
  }
  return 0;
}
