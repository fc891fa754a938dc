// tools/fetch_calib.hip — FETCH_SIZE / WRITE_SIZE calibration for the access widths k_bdpt_sample
// uses (MI355X_MICROARCH.md, HBM: FETCH_SIZE reads half the bytes of a 16-B/lane streaming read;
// "other access widths are uncalibrated"). Each kernel moves a known number of bytes of a 2 GiB
// buffer (8x the 256 MiB Infinity Cache, so the lines come from HBM):
//   k_read16  — 16 B per lane, a wave reads 1 KiB contiguous (the guide's reference case)
//   k_read4   — 4 B per lane, a wave reads 256 B contiguous (scratch / lane-interleaved dwords)
//   k_gather16— 16 B per lane at a random 128-B line (BVH node / primitive gathers)
//   k_gather64 / k_gather128 — 4 / 8 adjacent lanes read 16 B each of one random 128-B line (64 / 128
//               requested bytes per line): with the 16-B case they tell whether a gather moves the
//               whole line, together with TCC_BUBBLE / TCC_EA0_RDREQ and the kernels' durations
//               (a gather kernel cannot move 128 B per line faster than HBM allows)
//   k_write4  — 4 B per lane stores, 256 B per wave (scratch stores)
// Run under `rocprofv3 --pmc FETCH_SIZE --kernel-trace` (and WRITE_SIZE) and compare the counter
// with the bytes printed here. Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/bin/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_read16(const float4* __restrict__ a, size_t n, float* out) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  float s = 0;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) { float4 v = a[i]; s += v.x + v.y + v.z + v.w; }
  if (s == 12345.0f) out[0] = s;
}
__global__ void k_read4(const float* __restrict__ a, size_t n, float* out) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  float s = 0;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
  if (s == 12345.0f) out[0] = s;
}
__global__ void k_gather16(const float4* __restrict__ a, size_t nlines, size_t n, float* out) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  float s = 0;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t h = i * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    const size_t line = (size_t)(h % nlines);
    float4 v = a[line * 8];   // 128-B lines, 8 float4 each
    s += v.x + v.w;
  }
  if (s == 12345.0f) out[0] = s;
}
// `per` adjacent lanes share one random line: lane k of the group reads float4 k of it
template <int PER>
__global__ void k_gather_n(const float4* __restrict__ a, size_t nlines, size_t n, float* out) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  float s = 0;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t h = (i / PER) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    const size_t line = (size_t)(h % nlines);
    float4 v = a[line * 8 + (i % PER)];
    s += v.x + v.w;
  }
  if (s == 12345.0f) out[0] = s;
}
__global__ void k_write4(float* __restrict__ a, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (float)i;
}

int main() {
  const size_t bytes = (size_t)2 << 30;
  void* buf;
  float* out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 0, bytes));
  CK(hipDeviceSynchronize());
  const int grid = 256 * 32, block = 256;
  hipLaunchKernelGGL(k_read16, dim3(grid), dim3(block), 0, 0, (const float4*)buf, bytes / 16, out);
  printf("k_read16 requested_bytes %zu\n", bytes);
  hipLaunchKernelGGL(k_read4, dim3(grid), dim3(block), 0, 0, (const float*)buf, bytes / 4, out);
  printf("k_read4 requested_bytes %zu\n", bytes);
  const size_t ng = (size_t)64 << 20;   // 64 Mi gathers of 16 B = 1 GiB requested, 8 GiB of lines touched at most
  hipLaunchKernelGGL(k_gather16, dim3(grid), dim3(block), 0, 0, (const float4*)buf, bytes / 128, ng, out);
  printf("k_gather16 requested_bytes %zu lines_touched_max %zu\n", ng * 16, ng * 128);
  hipLaunchKernelGGL(k_gather_n<4>, dim3(grid), dim3(block), 0, 0, (const float4*)buf, bytes / 128, ng, out);
  printf("k_gather64 requested_bytes %zu lines %zu\n", ng * 16, ng / 4);
  hipLaunchKernelGGL(k_gather_n<8>, dim3(grid), dim3(block), 0, 0, (const float4*)buf, bytes / 128, ng, out);
  printf("k_gather128 requested_bytes %zu lines %zu\n", ng * 16, ng / 8);
  hipLaunchKernelGGL(k_write4, dim3(grid), dim3(block), 0, 0, (float*)buf, bytes / 4);
  printf("k_write4 written_bytes %zu\n", bytes);
  CK(hipDeviceSynchronize());
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
