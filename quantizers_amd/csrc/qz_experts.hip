// qz_experts.hip -- the per-expert GEMMs of a fixed-routing MoE forward, issued from C (host code).
//
// An AWQ grid over an MoE block re-runs the block 21 times with the routing fixed (moe_eager.py,
// planned form).  Every forward is two GEMMs per routed expert -- ~256 small hipBLASLt launches
// -- and issued one `torch.mm` at a time from Python the host, not the GPU, sets the pace
// (profiles/r03l_moe_breakdown.txt).  qz_expert_gemms issues a list of them in one call with
// the Python GIL released: for each (row range, expert) it makes the call torch.mm(x[rows],
// w[e].t(), out=out[rows]) makes -- the same hipBLASLt problem (column-major
// D[n, m] = op_T(A = w[e]) * op_N(B = x[rows]), f32 compute, bf16 in/out, alpha 1, beta 0), the
// heuristic's first algorithm under the same workspace limit -- so the same kernel and the same
// bits; the caller verifies that against torch.mm on each plan's first forward before using it.
//
// hipBLASLt is not linked: the functions are looked up in the copy already loaded in the process
// (PyTorch's bundled libhipblaslt, named by the caller through qz_expert_gemms_library), so there
// is exactly one copy of the library and its kernel selection is torch's.  Without it loaded the
// call returns QZ_ERR_UNAVAILABLE and qz_expert_gemms_status() says why.
//
// Threads: one mutex serialises the GEMM issue (one hipBLASLt handle per device, whose matmul is
// not documented thread-safe, and the problem cache): callers on several host threads / streams
// are safe and each one's launches stay in its own stream (tests/test_moe_eager.py, 4 threads).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/quantizers_amd.h"

namespace {

struct LtApi {
  decltype(&hipblasLtCreate) create = nullptr;
  decltype(&hipblasLtMatmulDescCreate) desc_create = nullptr;
  decltype(&hipblasLtMatmulDescSetAttribute) desc_set = nullptr;
  decltype(&hipblasLtMatrixLayoutCreate) layout_create = nullptr;
  decltype(&hipblasLtMatmulPreferenceCreate) pref_create = nullptr;
  decltype(&hipblasLtMatmulPreferenceSetAttribute) pref_set = nullptr;
  decltype(&hipblasLtMatmulPreferenceDestroy) pref_destroy = nullptr;
  decltype(&hipblasLtMatmulAlgoGetHeuristic) heuristic = nullptr;
  decltype(&hipblasLtMatmul) matmul = nullptr;
  bool ok = false;
};


// Which hipBLASLt: the copy already mapped into the process (PyTorch loads its bundled
// libhipblaslt.so as a dependency of libtorch_hip, RTLD_LOCAL, so it is not visible through
// RTLD_DEFAULT).  The caller names it: qz_expert_gemms_library(path) binds the library at `path`
// if -- and only if -- it is already loaded (RTLD_NOLOAD: this library never loads a second
// copy); without that call the first qz_expert_gemms binds the loaded object whose soname is
// "libhipblaslt.so.1" (ROCm's soname).  Every refusal leaves its reason in
// qz_expert_gemms_status().
std::mutex g_bind_mu;
void* g_lib = nullptr;
bool g_bound = false;
std::string g_status = "hipBLASLt not bound yet";
LtApi g_api;

template <class F>
bool sym(F& f, void* h, const char* name) {
  f = reinterpret_cast<F>(dlsym(h, name));
  if (!f) g_status = std::string("hipBLASLt symbol missing: ") + name;
  return f != nullptr;
}

void set_status(const std::string& m) {
  std::lock_guard<std::mutex> lk(g_bind_mu);
  g_status = m;
}

// caller holds g_bind_mu
int bind(const char* path) {
  dlerror();
  void* h = dlopen(path, RTLD_NOLOAD | RTLD_LAZY);
  if (!h) {
    const char* e = dlerror();
    g_status = std::string("hipBLASLt '") + path + "' is not loaded in this process" + (e ? std::string(": ") + e : "");
    return QZ_ERR_UNAVAILABLE;
  }
  LtApi a;
  bool ok = sym(a.create, h, "hipblasLtCreate") && sym(a.desc_create, h, "hipblasLtMatmulDescCreate") &&
            sym(a.desc_set, h, "hipblasLtMatmulDescSetAttribute") &&
            sym(a.layout_create, h, "hipblasLtMatrixLayoutCreate") &&
            sym(a.pref_create, h, "hipblasLtMatmulPreferenceCreate") &&
            sym(a.pref_set, h, "hipblasLtMatmulPreferenceSetAttribute") &&
            sym(a.pref_destroy, h, "hipblasLtMatmulPreferenceDestroy") &&
            sym(a.heuristic, h, "hipblasLtMatmulAlgoGetHeuristic") && sym(a.matmul, h, "hipblasLtMatmul");
  if (!ok) {
    dlclose(h);
    return QZ_ERR_UNAVAILABLE;
  }
  a.ok = true;
  g_api = a;
  g_lib = h;
  g_bound = true;
  g_status = std::string("bound: ") + path;
  return QZ_OK;
}

const LtApi& api() {
  std::lock_guard<std::mutex> lk(g_bind_mu);
  if (!g_bound) bind("libhipblaslt.so.1");
  return g_api;
}

// One GEMM problem: descriptors + the heuristic's algorithm, created once and kept (a few
// hundred distinct row counts per model; descriptors are small host objects).
struct Problem {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr;
  hipblasLtMatmulAlgo_t algo{};
};

struct Key {
  int dev;
  int64_t m, n, k, lda, ldb, ldc;
  uint64_t ws;
  bool operator==(const Key& o) const {
    return dev == o.dev && m == o.m && n == o.n && k == o.k && lda == o.lda && ldb == o.ldb && ldc == o.ldc &&
           ws == o.ws;
  }
};
struct KeyHash {
  size_t operator()(const Key& x) const {
    uint64_t h = 1469598103934665603ull;
    for (uint64_t v : {(uint64_t)x.dev, (uint64_t)x.m, (uint64_t)x.n, (uint64_t)x.k, (uint64_t)x.lda, (uint64_t)x.ldb,
                       (uint64_t)x.ldc, x.ws})
      h = (h ^ v) * 1099511628211ull;
    return (size_t)h;
  }
};

// One mutex serialises every qz_expert_gemms call: the calls share one hipBLASLt handle per device
// (whose matmul is not documented thread-safe) and the problem cache.  The product calls it from
// one host thread (an AWQ grid); a second caller waits for the first call's launches.
std::mutex g_mu;
std::unordered_map<int, hipblasLtHandle_t> g_handles;
std::unordered_map<Key, Problem, KeyHash> g_problems;

// Looks up (or builds) the problem; the caller holds g_mu.  Returns 0 or a QZ_ERR_* / positive status.
int problem(const LtApi& L, const Key& key, hipblasLtHandle_t* handle, const Problem** out) {
  auto hit = g_handles.find(key.dev);
  if (hit == g_handles.end()) {
    hipblasLtHandle_t h = nullptr;
    if (L.create(&h) != HIPBLAS_STATUS_SUCCESS) {
      set_status("hipblasLtCreate failed");
      return QZ_ERR_UNAVAILABLE;
    }
    hit = g_handles.emplace(key.dev, h).first;
  }
  *handle = hit->second;
  auto it = g_problems.find(key);
  if (it != g_problems.end()) {
    *out = &it->second;
    return QZ_OK;
  }
  Problem p;
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  if (L.desc_create(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS ||
      L.desc_set(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)) != HIPBLAS_STATUS_SUCCESS ||
      L.desc_set(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)) != HIPBLAS_STATUS_SUCCESS)
    return QZ_ERR_UNAVAILABLE;
  // column-major: A = w[e] seen as [k, n] (ld lda), op T; B = x[rows] seen as [k, m] (ld ldb);
  // C = D = out[rows] seen as [n, m] (ld ldc)
  if (L.layout_create(&p.a, HIP_R_16BF, key.k, key.n, key.lda) != HIPBLAS_STATUS_SUCCESS ||
      L.layout_create(&p.b, HIP_R_16BF, key.k, key.m, key.ldb) != HIPBLAS_STATUS_SUCCESS ||
      L.layout_create(&p.c, HIP_R_16BF, key.n, key.m, key.ldc) != HIPBLAS_STATUS_SUCCESS)
    return QZ_ERR_UNAVAILABLE;
  hipblasLtMatmulPreference_t pref = nullptr;
  if (L.pref_create(&pref) != HIPBLAS_STATUS_SUCCESS) return QZ_ERR_UNAVAILABLE;
  uint64_t ws = key.ws;
  hipblasLtMatmulHeuristicResult_t res{};
  int returned = 0;
  hipblasStatus_t st = L.pref_set(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
  if (st == HIPBLAS_STATUS_SUCCESS)
    st = L.heuristic(*handle, p.desc, p.a, p.b, p.c, p.c, pref, 1, &res, &returned);
  L.pref_destroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS || returned < 1 || res.state != HIPBLAS_STATUS_SUCCESS) {
    char msg[160];
    snprintf(msg, sizeof msg, "hipBLASLt heuristic: status %d, %d results (m %ld n %ld k %ld)", (int)st, returned,
             (long)key.m, (long)key.n, (long)key.k);
    set_status(msg);
    return QZ_ERR_UNAVAILABLE;
  }
  p.algo = res.algo;
  *out = &g_problems.emplace(key, p).first->second;
  return QZ_OK;
}

}  // namespace

extern "C" {

int qz_expert_gemms_library(const char* path) {
  if (!path) return QZ_ERR_NULL;
  std::lock_guard<std::mutex> lk(g_bind_mu);
  if (g_bound) {  // once per process: the same object again is fine, another one is refused
    void* h = dlopen(path, RTLD_NOLOAD | RTLD_LAZY);
    const bool same = h == g_lib;
    if (h) dlclose(h);
    if (!same) g_status = std::string("already bound to another hipBLASLt; refused ") + path;
    return same ? QZ_OK : QZ_ERR_FORMAT;
  }
  return bind(path);
}

const char* qz_expert_gemms_status(void) {
  static thread_local std::string copy;
  std::lock_guard<std::mutex> lk(g_bind_mu);
  copy = g_status;
  return copy.c_str();
}

int qz_expert_gemms(const void* x, int64_t ldx, const void* w, int64_t w_stride, int64_t ldw, int64_t n, int64_t k,
                    void* out, int64_t ldo, const int64_t* row0, const int64_t* row1, const int32_t* expert,
                    int32_t count, void* workspace, size_t workspace_bytes, qz_stream_t stream) {
  if (count < 0 || n <= 0 || k <= 0 || ldx < k || ldw < k || ldo < n) return QZ_ERR_SHAPE;
  if (count == 0) return QZ_OK;
  if (!x || !w || !out || !row0 || !row1 || !expert || (workspace_bytes && !workspace)) return QZ_ERR_NULL;
  const LtApi& L = api();
  if (!L.ok) return QZ_ERR_UNAVAILABLE;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return QZ_ERR_UNAVAILABLE;
  std::lock_guard<std::mutex> lock(g_mu);
  const float alpha = 1.0f, beta = 0.0f;
  const uint16_t* xb = (const uint16_t*)x;
  const uint16_t* wb = (const uint16_t*)w;
  uint16_t* ob = (uint16_t*)out;
  for (int32_t i = 0; i < count; ++i) {
    const int64_t m = row1[i] - row0[i];
    if (m < 0 || expert[i] < 0) return QZ_ERR_SHAPE;
    if (m == 0) continue;
    hipblasLtHandle_t h = nullptr;
    const Problem* p = nullptr;
    int rc = problem(L, Key{dev, m, n, k, ldw, ldx, ldo, (uint64_t)workspace_bytes}, &h, &p);
    if (rc) return rc;
    const hipblasStatus_t st =
        L.matmul(h, p->desc, &alpha, wb + (int64_t)expert[i] * w_stride, p->a, xb + row0[i] * ldx, p->b, &beta,
                 ob + row0[i] * ldo, p->c, ob + row0[i] * ldo, p->c, &p->algo, workspace, workspace_bytes,
                 (hipStream_t)stream);
    if (st != HIPBLAS_STATUS_SUCCESS) {
      set_status("hipblasLtMatmul status " + std::to_string((int)st) + " (m " + std::to_string((long)m) + ")");
      return QZ_ERR_UNAVAILABLE;
    }
  }
  return QZ_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// GEMM algorithm probe (tooling, not on the product path; scripts/gemm_algo_probe.py): the first
// `want` algorithms hipBLASLt's heuristic offers for torch.mm's problem out[m, n] = x[m, k] ·
// w[n, k]^T (bf16, f32 compute, the layout qz_expert_gemms uses), kept in a list; the script runs
// each one and compares its time and bits with torch.mm's.
namespace {
std::vector<hipblasLtMatmulAlgo_t> g_probe_algos;
Problem g_probe{};
}  // namespace

extern "C" {

int qz_gemm_probe_algos(int64_t m, int64_t n, int64_t k, size_t workspace_bytes, int32_t want, int32_t* n_algos) {
  const LtApi& L = api();
  if (!L.ok) return QZ_ERR_UNAVAILABLE;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return QZ_ERR_UNAVAILABLE;
  std::lock_guard<std::mutex> lock(g_mu);
  hipblasLtHandle_t h = nullptr;
  const Problem* p = nullptr;
  int rc = problem(L, Key{dev, m, n, k, k, k, n, (uint64_t)workspace_bytes}, &h, &p);
  if (rc) return rc;
  g_probe = *p;
  hipblasLtMatmulPreference_t pref = nullptr;
  if (L.pref_create(&pref) != HIPBLAS_STATUS_SUCCESS) return QZ_ERR_UNAVAILABLE;
  uint64_t ws = workspace_bytes;
  std::vector<hipblasLtMatmulHeuristicResult_t> res(want > 0 ? want : 1);
  int returned = 0;
  hipblasStatus_t st = L.pref_set(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
  if (st == HIPBLAS_STATUS_SUCCESS)
    st = L.heuristic(h, g_probe.desc, g_probe.a, g_probe.b, g_probe.c, g_probe.c, pref, (int)res.size(), res.data(),
                     &returned);
  L.pref_destroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS) return QZ_ERR_UNAVAILABLE;
  g_probe_algos.clear();
  for (int i = 0; i < returned; ++i)
    if (res[i].state == HIPBLAS_STATUS_SUCCESS) g_probe_algos.push_back(res[i].algo);
  *n_algos = (int32_t)g_probe_algos.size();
  return QZ_OK;
}

int qz_gemm_probe_run(int32_t i, const void* x, const void* w, void* out, void* workspace, size_t workspace_bytes,
                      qz_stream_t stream) {
  const LtApi& L = api();
  if (!L.ok || i < 0 || i >= (int32_t)g_probe_algos.size()) return QZ_ERR_SHAPE;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return QZ_ERR_UNAVAILABLE;
  std::lock_guard<std::mutex> lock(g_mu);
  const float alpha = 1.0f, beta = 0.0f;
  const hipblasStatus_t st = L.matmul(g_handles[dev], g_probe.desc, &alpha, w, g_probe.a, x, g_probe.b, &beta, out,
                                      g_probe.c, out, g_probe.c, &g_probe_algos[i], workspace, workspace_bytes,
                                      (hipStream_t)stream);
  return st == HIPBLAS_STATUS_SUCCESS ? QZ_OK : QZ_ERR_UNAVAILABLE;
}

}  // extern "C"
