// Main-loop microbenchmark for the conv engine (not product code): how fast can one
// 256x256-tile workgroup (8 waves, 128x64 per wave, 16x16x32 f16 MFMA) run
//   K1: MFMAs on register-resident fragments
//   K2: + 12 ds_read_b128 fragment reads per 32 MFMAs, one barrier per step
//   K3: K2 as ping-pong (second wave half one barrier behind, 2 barriers per step)
//   K4: K3 + LDS-DMA of 16 KiB per step from an L2-resident buffer (counted vmcnt)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mbench.hip -o /tmp/mbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 f16;
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gptr_t;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int TC = 8, TP = 4;

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int MODE>
__global__ __launch_bounds__(512, 1) void mloop(const f16* __restrict__ src, float* out, int steps, long long* clk) {
  __shared__ __attribute__((aligned(16))) char smem[163840];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  f32x4 acc[TC][TP];
  for (int a = 0; a < TC; ++a)
    for (int b = 0; b < TP; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fill LDS with something random-ish
  for (int i = threadIdx.x; i < 163840 / 16; i += 512) {
    f16x8 v;
    for (int j = 0; j < 8; ++j) v[j] = (f16)(((i * 8 + j) * 2654435761u >> 20) % 200 * 0.01f - 1.0f);
    *reinterpret_cast<f16x8*>(smem + i * 16) = v;
  }
  __syncthreads();
  f16x8 fa[TC], fb[TP];
  const int wr = wave / 4, wc = wave % 4;
  const int a_off = (wr * 128 + fr) * 64 + ((fq ^ ((fr >> 1) & 3)) << 4);
  const int b_off = 16384 + (wc * 64 + fr) * 64 + ((fq ^ ((fr >> 1) & 3)) << 4);
  for (int a = 0; a < TC; ++a) fa[a] = *reinterpret_cast<const f16x8*>(smem + a_off + a * 1024);
  for (int b = 0; b < TP; ++b) fb[b] = *reinterpret_cast<const f16x8*>(smem + b_off + b * 1024);
  const unsigned woff = (unsigned)(((wave * 2) * 16 + (lane >> 2)) * 4608) + ((lane & 3) << 4);   // 4608 B rows
  long long t0 = __builtin_amdgcn_s_memtime();
  const bool lag = wave >= 4;
  if (MODE >= 3 && lag) bar();
  for (int s = 0; s < steps; ++s) {
    const int slot = s & 3;
    if (MODE == 4) {
      const char* wb = reinterpret_cast<const char*>(src) + (s % 72) * 64;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        unsigned off = woff + i * 16 * 4608;
        asm volatile("" : "+v"(off));
        __builtin_amdgcn_global_load_lds((gptr_t)(wb + off), (lds_ptr_t)(smem + slot * 16384 + (wave * 2 + i) * 1024), 16, 0, 0);
      }
    }
    if (MODE >= 2) {
      const int so = (slot & 1) * 32768;
      for (int a = 0; a < TC; ++a) fa[a] = *reinterpret_cast<const f16x8*>(smem + so + a_off + a * 1024);
      for (int b = 0; b < TP; ++b) fb[b] = *reinterpret_cast<const f16x8*>(smem + so + b_off + b * 1024);
    }
    if (MODE == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    if (MODE >= 2) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (MODE >= 2) bar();
#pragma unroll
    for (int a = 0; a < TC; ++a)
#pragma unroll
      for (int b = 0; b < TP; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[a], fb[b], acc[a][b], 0, 0, 0);
    if (MODE >= 3) bar();
  }
  if (MODE >= 3 && !lag) bar();
  long long t1 = __builtin_amdgcn_s_memtime();
  float sum = 0.f;
  for (int a = 0; a < TC; ++a)
    for (int b = 0; b < TP; ++b) sum += acc[a][b][0] + acc[a][b][1] + acc[a][b][2] + acc[a][b][3];
  out[blockIdx.x * 512 + threadIdx.x] = sum;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(int nwg, int steps, const f16* src, float* out, long long* clk) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(mloop<MODE>, dim3(nwg), dim3(512), 0, 0, src, out, steps, clk);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  const int reps = 10;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(mloop<MODE>, dim3(nwg), dim3(512), 0, 0, src, out, steps, clk);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  std::vector<long long> c(nwg);
  CHECK(hipMemcpy(c.data(), clk, nwg * 8, hipMemcpyDeviceToHost));
  double avgc = 0;
  for (auto v : c) avgc += v;
  avgc /= nwg;
  const double flop = 2.0 * 256 * 256 * 32 * (double)steps * nwg;
  // s_memtime counts the shader clock: cycles per step vs the MFMA bound of 1024
  printf("mode %d nwg %d steps %d: %.3f ms  %.1f TFLOP/s  cycles/step %.0f (MFMA bound 1024)  clock %.2f GHz\n", MODE,
         nwg, steps, ms, flop / (ms * 1e-3) / 1e12, avgc / steps, avgc / (ms * 1e-3) / 1e9);
}

int main(int argc, char** argv) {
  const int nwg = argc > 1 ? atoi(argv[1]) : 256;
  const int steps = argc > 2 ? atoi(argv[2]) : 2000;
  f16* src; float* out; long long* clk;
  CHECK(hipMalloc(&src, 256 * 4608 * 2));
  CHECK(hipMemset(src, 0x3c, 256 * 4608 * 2));
  CHECK(hipMalloc(&out, nwg * 512 * 4));
  CHECK(hipMalloc(&clk, nwg * 8));
  run<1>(nwg, steps, src, out, clk);
  run<2>(nwg, steps, src, out, clk);
  run<3>(nwg, steps, src, out, clk);
  run<4>(nwg, steps, src, out, clk);
  return 0;
}
