// Counter calibration kernels (kernel studies only, never loaded by the product): known byte counts in the
// access shapes of the K14 evaluation, to read rocprofv3 FETCH_SIZE / WRITE_SIZE against.  Built by
// tools/calib.sh into tools/libcalib.so; driven by tools/calib.py.
//   read16   : lane-contiguous 16-B loads (global_load_dwordx4), grid-stride   -- the guide's "half-count" shape
//   read_prep: the prep's fp64 row shape: lane L loads elements 4L..4L+3 as two 16-B double2 loads, 256-element
//              strides (load4d in cmve_internal.h)
//   write8   : 8-B stores per lane (the prep's fp16 plane stores: cmve_u16x4)
//   write16  : 16-B stores per lane
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void read16_kernel(const double2* __restrict__ p, int64_t n2, double* __restrict__ sink) {
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x) {
    const double2 v = p[i];
    acc += v.x + v.y;
  }
  if (acc == 12345.678) sink[0] = acc;  // never true for the zero-filled buffers: keeps the loads
}

// rows of 1024 doubles, one wave per row (the eval prep's register path: 4 x (2 x double2) per lane)
__global__ void read_prep_kernel(const double* __restrict__ p, int64_t rows, double* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const double* x = p + row * 1024;
  double acc = 0.0;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const double2 a = *(const double2*)(x + lane * 4 + 256 * m), b = *(const double2*)(x + lane * 4 + 256 * m + 2);
    acc += a.x + a.y + b.x + b.y;
  }
  if (acc == 12345.678) sink[0] = acc;
}

typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

__global__ void write8_kernel(u16x4* __restrict__ p, int64_t n) {
  const u16x4 z = {1, 2, 3, 4};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = z;
}

__global__ void write16_kernel(float4* __restrict__ p, int64_t n) {
  const float4 z = {1.f, 2.f, 3.f, 4.f};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = z;
}

extern "C" int calib_read16(const void* p, int64_t bytes, double* sink, void* stream) {
  hipLaunchKernelGGL(read16_kernel, dim3(2048), dim3(256), 0, (hipStream_t)stream, (const double2*)p, bytes / 16, sink);
  return (int)hipGetLastError();
}
extern "C" int calib_read_prep(const void* p, int64_t bytes, double* sink, void* stream) {
  const int64_t rows = bytes / 8192;
  hipLaunchKernelGGL(read_prep_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     (const double*)p, rows, sink);
  return (int)hipGetLastError();
}
extern "C" int calib_write8(void* p, int64_t bytes, void* stream) {
  hipLaunchKernelGGL(write8_kernel, dim3(2048), dim3(256), 0, (hipStream_t)stream, (u16x4*)p, bytes / 8);
  return (int)hipGetLastError();
}
extern "C" int calib_write16(void* p, int64_t bytes, void* stream) {
  hipLaunchKernelGGL(write16_kernel, dim3(2048), dim3(256), 0, (hipStream_t)stream, (float4*)p, bytes / 16);
  return (int)hipGetLastError();
}
