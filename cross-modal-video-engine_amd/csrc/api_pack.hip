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

namespace cmve {

static thread_local std::string g_last_error;

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

// ---------------------------------------------------------------------------
// K1: pack
// ---------------------------------------------------------------------------
template <typename T>
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
    for (int64_t k = lane; k < d_pad; k += 64) {
      hrow[k] = 0;
      if (lrow) lrow[k] = 0;
      if (frow) frow[k] = 0;
    }
    if (lane == 0) {
      inv_norm[row] = 0.0;
      err_hi[row] = 0.f;
      err_hilo[row] = 0.f;
      if (err_h16) err_h16[row] = 0.f;
    }
    return;
  }
  const T* x = raw + row * ld;
  double ss = 0.0;
  for (int64_t k = lane; k < d; k += 64) {
    double v = (double)x[k];
    ss = fma(v, v, ss);
  }
  ss = wave_sum(ss);
  const double nrm = sqrt(ss);
  // eps == 0: LINAS l2norm (X / norm, NaN on a zero row); eps > 0: F.normalize
  const double inv = (flags & CMVE_PACK_RAW) ? 1.0 : (eps > 0.0 ? 1.0 / fmax(nrm, eps) : 1.0 / nrm);
  double e1 = 0.0, e2 = 0.0, e3 = 0.0;
  for (int64_t k = lane; k < d_pad; k += 64) {
    if (k < d) {
      const double xh = (double)x[k] * inv;
      if (frow) {
        const _Float16 hf16 = (_Float16)xh;  // RNE from fp64
        const double r3 = xh - (double)hf16;
        e3 = fma(r3, r3, e3);
        frow[k] = __builtin_bit_cast(uint16_t, hf16);
      }
      const float xf = (float)xh;
      const uint16_t h = f2bf(xf);
      const float hf = bf2f(h);
      const uint16_t l = f2bf(xf - hf);
      const double r1 = xh - (double)hf;
      const double r2 = r1 - (double)bf2f(l);
      e1 = fma(r1, r1, e1);
      e2 = fma(r2, r2, e2);
      hrow[k] = h;
      if (lrow) lrow[k] = l;
    } else {
      hrow[k] = 0;
      if (lrow) lrow[k] = 0;
      if (frow) frow[k] = 0;
    }
  }
  e1 = wave_sum(e1);
  e2 = wave_sum(e2);
  e3 = wave_sum(e3);
  if (lane == 0) {
    inv_norm[row] = inv;
    // sqrt rounding + the fp64 error of x*inv itself (~1e-16 per element) -> small slack
    const float b1 = f32_round_up(sqrt(e1) * (1.0 + 1e-9) + 1e-12);
    const float b2 = f32_round_up(sqrt(e2) * (1.0 + 1e-9) + 1e-12);
    err_hi[row] = b1;
    err_hilo[row] = b2;
    if (b1 == b1) atomicMax((int*)&err_max[0], __float_as_int(b1));  // non-negative floats order as ints
    if (b2 == b2) atomicMax((int*)&err_max[1], __float_as_int(b2));
    if (err_h16) {
      const float b3 = f32_round_up(sqrt(e3) * (1.0 + 1e-9) + 1e-12);
      err_h16[row] = b3;
      if (b3 == b3) atomicMax((int*)&err_max[2], __float_as_int(b3));
    }
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
  CMVE_HIP(hipMemsetAsync(r->err_max, 0, 3 * sizeof(float), h->stream));
  dim3 grid((unsigned)((r->n_pad + 3) / 4)), block(256);
  if (r->raw_dtype == CMVE_F32)
    hipLaunchKernelGGL(pack_rows_kernel<float>, grid, block, 0, h->stream, (const float*)r->raw, r->raw_ld, r->n,
                       r->d, r->n_pad, r->d_pad, r->eps, r->flags, r->hi, r->lo, r->h16, r->inv_norm, r->err_hi, r->err_hilo,
                       r->err_h16, r->err_max);
  else if (r->raw_dtype == CMVE_F64)
    hipLaunchKernelGGL(pack_rows_kernel<double>, grid, block, 0, h->stream, (const double*)r->raw, r->raw_ld, r->n,
                       r->d, r->n_pad, r->d_pad, r->eps, r->flags, r->hi, r->lo, r->h16, r->inv_norm, r->err_hi, r->err_hilo,
                       r->err_h16, r->err_max);
  else {
    set_error("cmve_pack_rows: raw_dtype must be CMVE_F32 or CMVE_F64");
    return CMVE_E_INVALID;
  }
  return check_launch("pack_rows");
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
