// Handle / error plumbing and K1 (row L2 normalisation + split-bf16 packing).
//
// K1 replaces LINAS-engine/evaluation.py:10-14 and LINAS-engine/model.py:35-40
// (l2norm, no epsilon) and F.normalize (eps 1e-12) at MultiFusion/src/combiner.py:134,180
// and MultiFusion/src/validate.py:55.  One wave per row; the norm and the residual
// bounds are accumulated in fp64 so the error bound used by the rank epilogue is
// rigorous.
#include "cmve_internal.h"
#include <stdarg.h>
#include <stdio.h>
#include <atomic>

namespace cmve {

static thread_local std::string g_last_error;
thread_local LaunchEv g_launch_ev;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: kernel launch failed: %s", what, hipGetErrorString(e));
    return CMVE_E_HIP;
  }
  return CMVE_OK;
}

int device_cus() {
  // one slot per device ordinal: a host thread per GPU may ask concurrently (relaxed atomics: the value
  // is a pure function of the device, so a racing double query stores the same number)
  static std::atomic<int> cus[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  int c = cus[dev].load(std::memory_order_relaxed);
  if (!c) {
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    cus[dev].store(c, std::memory_order_relaxed);
  }
  return c;
}

// ---------------------------------------------------------------------------
// K1: pack
// ---------------------------------------------------------------------------
// One wave per row.  VEC: fp32 rows with d % 4 == 0 and 16-B aligned rows -- each lane moves 4
// consecutive elements (16-B loads, 8-B plane stores); otherwise one element per lane step.
// (row_sumsq / pack_row_planes, cmve_internal.h: the K14 evaluation kernel packs with the same code)
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void pack_rows_kernel(const T* __restrict__ raw, int64_t ld, int64_t n,
                                                        int64_t d, int64_t n_pad, int64_t d_pad, double eps, int flags,
                                                        uint16_t* __restrict__ hi, uint16_t* __restrict__ lo,
                                                        uint16_t* __restrict__ h16, double* __restrict__ inv_norm,
                                                        float* __restrict__ err_hi, float* __restrict__ err_hilo,
                                                        float* __restrict__ err_h16, float* __restrict__ err_max) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n_pad) return;
  uint16_t* hrow = hi + row * d_pad;
  uint16_t* lrow = lo ? lo + row * d_pad : nullptr;
  uint16_t* frow = h16 ? h16 + row * d_pad : nullptr;
  if (row >= n) {  // padding rows: zero vectors, zero bounds
    pack_pad_row(hrow, lrow, frow, d_pad, lane);
    if (lane == 0) {
      inv_norm[row] = 0.0;
      err_hi[row] = 0.f;
      err_hilo[row] = 0.f;
      if (err_h16) err_h16[row] = 0.f;
    }
    return;
  }
  const T* x = raw + row * ld;
  // eps == 0: LINAS l2norm (X / norm, NaN on a zero row); eps > 0: F.normalize
  const double inv = row_inv_norm(row_sumsq<T>(x, d, VEC, lane), eps, flags);
  float b1, b2, b3;
  pack_row_planes<T>(x, d, d_pad, VEC, inv, hrow, lrow, frow, lane, b1, b2, b3);
  if (lane == 0) {
    inv_norm[row] = inv;
    err_hi[row] = b1;
    err_hilo[row] = b2;
    if (err_h16) err_h16[row] = b3;
  }
}

// err_max[s] = max over rows of the per-row bounds (NaN rows -- zero rows at eps == 0 -- skipped).
// One block: a same-address atomic per row serialises at one L2 channel (~30 ns each).
__global__ __launch_bounds__(1024) void err_max_kernel(const float* __restrict__ e0, const float* __restrict__ e1,
                                                       const float* __restrict__ e2, int64_t n,
                                                       float* __restrict__ err_max) {
  __shared__ float part[3][16];
  float m0 = 0.f, m1 = 0.f, m2 = 0.f;  // bounds are >= 0
  for (int64_t i = threadIdx.x; i < n; i += 1024) {
    m0 = fmaxf(m0, e0[i]);  // fmaxf drops a NaN operand
    m1 = fmaxf(m1, e1[i]);
    if (e2) m2 = fmaxf(m2, e2[i]);
  }
  m0 = wave_max(m0);
  m1 = wave_max(m1);
  m2 = wave_max(m2);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    part[0][w] = m0;
    part[1][w] = m1;
    part[2][w] = m2;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    float m = 0.f;
    for (int k = 0; k < 16; ++k) m = fmaxf(m, part[threadIdx.x][k]);
    err_max[threadIdx.x] = m;
  }
}

// y = x / max(||x||, eps)   (eps == 0 -> x / ||x||)
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void l2norm_kernel(const TI* __restrict__ x, int64_t ldx, TO* __restrict__ y,
                                                     int64_t ldy, int64_t n, int64_t d, double eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const TI* xr = x + row * ldx;
  double ss = 0.0;
  for (int64_t k = lane; k < d; k += 64) {
    double v = (double)xr[k];
    ss = fma(v, v, ss);
  }
  ss = wave_sum(ss);
  const double nrm = sqrt(ss);
  const double den = eps > 0.0 ? fmax(nrm, eps) : nrm;
  TO* yr = y + row * ldy;
  for (int64_t k = lane; k < d; k += 64) yr[k] = (TO)((double)xr[k] / den);
}

int ensure_scratch(cmve_handle* h, size_t bytes) {
  if (h->scratch_bytes >= bytes) return CMVE_OK;
  if (h->scratch) {
    CMVE_HIP(hipStreamSynchronize(h->stream));
    CMVE_HIP(hipFree(h->scratch));
    h->scratch = nullptr;
    h->scratch_bytes = 0;
  }
  const size_t grown = std::max(bytes, (size_t)1 << 20);
  CMVE_HIP(hipMalloc(&h->scratch, grown));
  h->scratch_bytes = grown;
  return CMVE_OK;
}
}  // namespace cmve

using namespace cmve;

extern "C" {

int cmve_abi_version(void) { return CMVE_ABI_VERSION; }

const char* cmve_last_error(void) { return g_last_error.c_str(); }

int cmve_create(int device, void* hip_stream, cmve_handle_t* out) {
  CMVE_REQUIRE(out != nullptr, "cmve_create: out is NULL");
  int count = 0;
  CMVE_HIP(hipGetDeviceCount(&count));
  CMVE_REQUIRE(device >= 0 && device < count, "cmve_create: device %d out of range (%d devices)", device, count);
  cmve_handle* h = new cmve_handle;
  h->device = device;
  h->stream = (hipStream_t)hip_stream;
  *out = h;
  return CMVE_OK;
}

int cmve_set_stream(cmve_handle_t h, void* hip_stream) {
  CMVE_REQUIRE(h != nullptr, "cmve_set_stream: NULL handle");
  h->stream = (hipStream_t)hip_stream;
  return CMVE_OK;
}


int cmve_destroy(cmve_handle_t h) {
  if (h) {
    dist_release(h);
    if (h->scratch) (void)hipFree(h->scratch);
    for (hipEvent_t e : h->ev)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : h->tev)
      if (e) (void)hipEventDestroy(e);
    for (auto& slot : h->eval_ev)
      for (hipEvent_t e : slot)
        if (e) (void)hipEventDestroy(e);
    for (auto& slot : h->eval_kev)
      for (hipEvent_t e : slot)
        if (e) (void)hipEventDestroy(e);
    if (h->aux) (void)hipStreamDestroy(h->aux);
  }
  delete h;
  return CMVE_OK;
}

int cmve_pack_size(int64_t n, int64_t d, int64_t* n_pad, int64_t* d_pad) {
  CMVE_REQUIRE(n >= 0 && d > 0 && n_pad && d_pad, "cmve_pack_size: bad arguments n=%lld d=%lld", (long long)n,
               (long long)d);
  *n_pad = ((n + CMVE_ROW_ALIGN - 1) / CMVE_ROW_ALIGN) * CMVE_ROW_ALIGN;
  if (*n_pad == 0) *n_pad = CMVE_ROW_ALIGN;
  *d_pad = ((d + CMVE_DIM_ALIGN - 1) / CMVE_DIM_ALIGN) * CMVE_DIM_ALIGN;
  return CMVE_OK;
}

int cmve_pack_rows(cmve_handle_t h, cmve_rows_t* r) {
  CMVE_REQUIRE(h && r, "cmve_pack_rows: NULL argument");
  int64_t np_, dp_;
  if (cmve_pack_size(r->n, r->d, &np_, &dp_) != CMVE_OK) return CMVE_E_INVALID;
  CMVE_REQUIRE(r->n_pad == np_ && r->d_pad == dp_, "cmve_pack_rows: n_pad/d_pad must be %lld/%lld", (long long)np_,
               (long long)dp_);
  CMVE_REQUIRE(r->hi && r->inv_norm && r->err_hi && r->err_hilo && r->err_max, "cmve_pack_rows: NULL output");
  CMVE_REQUIRE(r->n == 0 || r->raw, "cmve_pack_rows: raw is NULL");
  CMVE_REQUIRE(r->raw_ld >= r->d, "cmve_pack_rows: raw_ld < d");
  CMVE_REQUIRE(r->eps >= 0.0, "cmve_pack_rows: eps < 0");
  CMVE_REQUIRE((r->h16 == nullptr) == (r->err_h16 == nullptr), "cmve_pack_rows: h16 and err_h16 go together");
  dim3 grid((unsigned)((r->n_pad + 3) / 4)), block(256);
  const bool vec = r->n == 0 || (r->raw_dtype == CMVE_F32 ? rows_vec4((const float*)r->raw, r->d, r->raw_ld)
                                                           : rows_vec4((const double*)r->raw, r->d, r->raw_ld));
#define PACK(T, V)                                                                                                   \
  hipLaunchKernelGGL((pack_rows_kernel<T, V>), grid, block, 0, h->stream, (const T*)r->raw, r->raw_ld, r->n, r->d, \
                     r->n_pad, r->d_pad, r->eps, r->flags, r->hi, r->lo, r->h16, r->inv_norm, r->err_hi, r->err_hilo,  \
                     r->err_h16, r->err_max)
  if (r->raw_dtype == CMVE_F32 && vec)
    PACK(float, true);
  else if (r->raw_dtype == CMVE_F32)
    PACK(float, false);
  else if (r->raw_dtype == CMVE_F64 && vec)
    PACK(double, true);
  else if (r->raw_dtype == CMVE_F64)
    PACK(double, false);
  else {
    set_error("cmve_pack_rows: raw_dtype must be CMVE_F32 or CMVE_F64");
    return CMVE_E_INVALID;
  }
#undef PACK
  int st = check_launch("pack_rows");
  if (st) return st;
  if (r->flags & CMVE_PACK_RAW) {  // GEMM operands of cmve_linear / cmve_sim_store: no score bound
    CMVE_HIP(hipMemsetD32Async((hipDeviceptr_t)r->err_max, 0x7f800000u, 3, h->stream));  // +inf
    return CMVE_OK;
  }
  hipLaunchKernelGGL(err_max_kernel, dim3(1), dim3(1024), 0, h->stream, r->err_hi, r->err_hilo, r->err_h16, r->n,
                     r->err_max);
  return check_launch("pack_rows/err_max");
}

int cmve_l2norm_rows(cmve_handle_t h, const void* x, int32_t x_dtype, int64_t ldx, void* y, int32_t y_dtype,
                     int64_t ldy, int64_t n, int64_t d, double eps) {
  CMVE_REQUIRE(h && x && y, "cmve_l2norm_rows: NULL argument");
  CMVE_REQUIRE(n >= 0 && d > 0 && ldx >= d && ldy >= d, "cmve_l2norm_rows: bad shape");
  if (n == 0) return CMVE_OK;
  dim3 grid((unsigned)((n + 3) / 4)), block(256);
#define L2N(TI, TO)                                                                                             \
  hipLaunchKernelGGL((l2norm_kernel<TI, TO>), grid, block, 0, h->stream, (const TI*)x, ldx, (TO*)y, ldy, n, d, \
                     eps)
  if (x_dtype == CMVE_F32 && y_dtype == CMVE_F32) L2N(float, float);
  else if (x_dtype == CMVE_F32 && y_dtype == CMVE_F64) L2N(float, double);
  else if (x_dtype == CMVE_F64 && y_dtype == CMVE_F32) L2N(double, float);
  else if (x_dtype == CMVE_F64 && y_dtype == CMVE_F64) L2N(double, double);
  else {
    set_error("cmve_l2norm_rows: dtypes must be CMVE_F32/CMVE_F64");
    return CMVE_E_INVALID;
  }
#undef L2N
  return check_launch("l2norm_rows");
}

}  // extern "C"
