// A C++ caller of the library's C ABI (include/quantizers_amd.h) with plain hipMalloc'd
// buffers -- what a non-Python integration looks like -- checked against the plain-C oracle
// (oracle/quant_ref.c, TEST INFRASTRUCTURE ONLY).  Built and run by tests/test_c_abi_gpu.py:
//   hipcc --offload-arch=gfx950 c_abi_demo.cpp -I include -L quantizers_amd -lquantizers_amd
//         -L oracle/build -lquant_ref
// Exit code 0 = bit-identical packed int4 words and bf16 scales for W[rows, cols], g128.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "quantizers_amd.h"

extern "C" int qref_int_sym_group_pack(const uint16_t* w, int64_t R, int64_t C, int bits, int g, int32_t* packed,
                                       uint16_t* scale);

static uint16_t to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

int main(int argc, char** argv) {
  const int64_t R = argc > 1 ? atoll(argv[1]) : 1024, C = argc > 2 ? atoll(argv[2]) : 4096;
  const int g = 128;
  std::vector<uint16_t> w(R * C);
  uint64_t st = 0x9E3779B97F4A7C15ull;
  for (auto& x : w) {  // deterministic pseudo-normal-ish weights (sum of uniforms), sigma ~0.02
    float acc = 0.f;
    for (int k = 0; k < 4; ++k) {
      st ^= st << 13; st ^= st >> 7; st ^= st << 17;
      acc += (float)(st >> 40) / (float)(1ull << 24) - 0.5f;
    }
    x = to_bf16(acc * 0.035f);
  }
  qz_args a = {4, QZ_INT, 1, QZ_GROUP, g, 0, 0, QZ_SCALE_NATIVE};
  void *dw, *dq, *ds, *dws;
  const size_t ws = qz_quantize_workspace_size(1, R, C, &a);
  if (hipMalloc(&dw, R * C * 2) || hipMalloc(&dq, R * C / 2) || hipMalloc(&ds, R * (C / g) * 2) ||
      hipMalloc(&dws, ws + 256))
    return 10;
  hipStream_t s;
  if (hipStreamCreate(&s)) return 11;
  if (hipMemcpy(dw, w.data(), R * C * 2, hipMemcpyHostToDevice)) return 12;
  int rc = qz_quantize(dw, 1, R, C, C, R * C, &a, QZ_OUT_PACKED_INT32, dq, ds, nullptr, nullptr, dws, ws + 256, s);
  if (rc) {
    std::fprintf(stderr, "qz_quantize: %s\n", qz_strerror(rc));
    return 13;
  }
  if (hipStreamSynchronize(s)) return 14;
  std::vector<int32_t> q(R * C / 8), qr(R * C / 8);
  std::vector<uint16_t> sc(R * (C / g)), sr(R * (C / g));
  if (hipMemcpy(q.data(), dq, q.size() * 4, hipMemcpyDeviceToHost) ||
      hipMemcpy(sc.data(), ds, sc.size() * 2, hipMemcpyDeviceToHost))
    return 15;
  qref_int_sym_group_pack(w.data(), R, C, 4, g, qr.data(), sr.data());
  const bool ok = std::memcmp(q.data(), qr.data(), q.size() * 4) == 0 && std::memcmp(sc.data(), sr.data(), sc.size() * 2) == 0;
  std::printf("qz_version %d, [%lld, %lld] int4 g%d via the C ABI: %s\n", qz_version(), (long long)R, (long long)C, g,
              ok ? "bit-identical to the C oracle" : "MISMATCH");
  hipFree(dw); hipFree(dq); hipFree(ds); hipFree(dws); hipStreamDestroy(s);
  return ok ? 0 : 1;
}
