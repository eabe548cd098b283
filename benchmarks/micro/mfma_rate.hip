// Calibration: back-to-back v_mfma_f32_16x16x32_bf16 on NA AGPR accumulators with NR
// ds_read_b128 fragment reads spread between them (the conv_direct tap pattern), NW waves per
// block (one block per CU by LDS).  Prints us per launch and achieved TFLOP/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NA, int NR, int NW, int NB>
__global__ void __launch_bounds__(64 * NW, 1) k(float *out, int iters) {
  __shared__ __attribute__((aligned(1024))) char smem[128 * 1024];
  f32x4 acc[NA];
  for (int i = 0; i < NA; ++i) { acc[i] = f32x4{0.f, 0.f, 0.f, 0.f}; asm volatile("" : "+a"(acc[i])); }
  constexpr int NAa = NB, NBb = NA / NB;  // NA = NAa (W frags) x NBb (x frags)
  bf16x8 a[NAa], b[NBb];
  const int lane = threadIdx.x & 63;
  for (int i = 0; i < NAa; ++i) a[i] = *reinterpret_cast<const bf16x8 *>(smem + 16 * lane + 1024 * i);
  for (int i = 0; i < NBb; ++i) b[i] = *reinterpret_cast<const bf16x8 *>(smem + 16 * lane + 1024 * (NAa + i));
  constexpr int RS = NR > 0 ? (NA / NR > 0 ? NA / NR : 1) : 1;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < NA; ++q) {
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[q]) : "v"(a[q % NAa]), "v"(b[q / NAa]));
      if constexpr (NR > 0) {
        if (q % RS == RS - 1 && q / RS < NR) {
          const int r = q / RS;
          const int off = 16 * lane + 1024 * ((it * 7 + r) & 63);
          if (r < NAa) a[r] = *reinterpret_cast<const bf16x8 *>(smem + off);
          else if (r - NAa < NBb) b[r - NAa] = *reinterpret_cast<const bf16x8 *>(smem + off);
        }
      }
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  float s = 0.f;
  for (int i = 0; i < NA; ++i) { asm volatile("" : "+a"(acc[i])); s += acc[i][0] + acc[i][3]; }
  out[blockIdx.x * 64 * NW + threadIdx.x] = s;
}

template <int NA, int NR, int NW, int NB>
void run(float *out, int iters, const char *name) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k<NA, NR, NW, NB>), dim3(256), dim3(64 * NW), 0, 0, out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  const double flop = 256.0 * NW * iters * NA * 16 * 16 * 32 * 2;
  printf("%-34s NA=%2d NR=%2d NW=%d  reads/MFMA %.2f  %8.1f us  %5.0f TFLOP/s\n", name, NA, NR, NW, (double)NR / NA,
         best * 1e3, flop / (best * 1e-3) / 1e12);
}

int main(int argc, char **argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  float *out;
  (void)hipMalloc(&out, 256 * 1024 * 4);
  run<24, 0, 4, 4>(out, iters, "mfma only");
  run<24, 10, 4, 4>(out, iters, "conv_direct 6x4 tile");
  run<24, 10, 8, 4>(out, iters / 2, "6x4 tile, 2 waves/SIMD");
  run<12, 7, 8, 4>(out, iters, "3x4 tile, 2 waves/SIMD");
  run<48, 14, 4, 8>(out, iters / 2, "6x8 tile");
  run<48, 16, 4, 4>(out, iters / 2, "12x4 tile");
  run<64, 16, 4, 8>(out, iters / 2, "8x8 tile");
  run<32, 12, 4, 4>(out, iters / 2, "8x4 tile");
  run<32, 12, 8, 4>(out, iters / 4, "8x4 tile, 2 waves/SIMD");
  return 0;
}
