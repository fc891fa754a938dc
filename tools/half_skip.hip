// Probe: does a wave64 VALU instruction on MI355X (SIMD-32, two passes per instruction) cost less
// when one 32-lane half of the wave has no active lane? Each wave runs the same FMA loop (8
// independent chains, so the loop is issue-bound, 4 waves per SIMD) under different exec masks;
// the kernel times are compared. Build: hipcc --offload-arch=gfx950 -O3 tools/half_skip.hip -o
// tools/bin/half_skip (and with -fno-slp-vectorize: tools/bin/half_skip_scalar, plain v_fma_f32)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(256) void k_fma(float* out, int iters, uint64_t mask) {
  const int lane = threadIdx.x & 63;
  if (!((mask >> lane) & 1)) return;
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  const float m = 1.0000001f, c = 0.999f;
  for (int i = 0; i < iters; i++) {
    a0 = fmaf(a0, m, c); a1 = fmaf(a1, m, c); a2 = fmaf(a2, m, c); a3 = fmaf(a3, m, c);
    a4 = fmaf(a4, m, c); a5 = fmaf(a5, m, c); a6 = fmaf(a6, m, c); a7 = fmaf(a7, m, c);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

int main() {
  const int blocks = 256 * 4, threads = 256, iters = 1 << 16;   // 16 waves per CU: 4 per SIMD
  float* out;
  if (hipMalloc(&out, sizeof(float) * blocks * threads) != hipSuccess) return 1;
  struct { const char* name; uint64_t mask; } cases[] = {
      {"all 64 lanes", ~0ull},
      {"lanes 0-31 (low half only)", 0xffffffffull},
      {"lanes 32-63 (high half only)", 0xffffffff00000000ull},
      {"lanes 0-15", 0xffffull},
      {"lanes 0-7", 0xffull},
      {"lanes 0-3", 0xfull},
      {"lanes 0-1", 0x3ull},
      {"lane 0 only", 1ull},
      {"lane 5 only", 1ull << 5},
      {"lanes 0 and 32 (one per half)", 1ull | (1ull << 32)},
      {"every 8th lane (8 lanes)", 0x0101010101010101ull},
      {"every 4th lane (16 lanes)", 0x1111111111111111ull},
      {"even lanes (both halves)", 0x5555555555555555ull},
      {"no lane", 0ull},
  };
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  k_fma<<<blocks, threads>>>(out, iters, ~0ull);   // warm-up
  (void)hipDeviceSynchronize();
  for (int rep = 0; rep < 2; rep++)
    for (auto& cs : cases) {
      (void)hipEventRecord(e0);
      k_fma<<<blocks, threads>>>(out, iters, cs.mask);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      // VALU instructions per wave: 8 FMAs per iteration (+ loop overhead)
      const double waves = (double)blocks * threads / 64, inst = waves * 8.0 * iters;
      const double cyc_per_inst = ms * 1e-3 * 2.4e9 * 1024 / inst;   // 1024 SIMDs, ~2.4 GHz
      printf("%-32s %8.3f ms  ~%.2f SIMD cycles per wave64 FMA\n", cs.name, ms, cyc_per_inst);
    }
  (void)hipFree(out);
  return 0;
}
