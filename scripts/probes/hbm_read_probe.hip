#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#define GA __attribute__((address_space(1)))
#define LA __attribute__((address_space(3)))
typedef float f32x4 __attribute__((ext_vector_type(4)));

// register path: each lane 16B loads, G loads in flight per group, grid-stride by chunks
template <int G, bool NT>
__global__ __launch_bounds__(256) void reg_read(const f32x4* __restrict__ src, int64_t n, uint32_t* out) {
  uint32_t x = 0;
  const int64_t stride = (int64_t)gridDim.x * 256 * G;
  for (int64_t base = (int64_t)blockIdx.x * 256 * G; base < n; base += stride) {
    f32x4 v[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      int64_t i = base + g * 256 + threadIdx.x;
      if (i < n) v[g] = NT ? __builtin_nontemporal_load(src + i) : src[i]; else v[g] = f32x4{0,0,0,0};
    }
#pragma unroll
    for (int g = 0; g < G; ++g) x ^= __float_as_uint(v[g].x) ^ __float_as_uint(v[g].y) ^ __float_as_uint(v[g].z) ^ __float_as_uint(v[g].w);
  }
  if (x == 0x12345678u) out[blockIdx.x] = x;
}

// LDS-DMA path: each wave streams its own 1 KiB pieces into a private LDS ring (G per group,
// double buffered), waits with vmcnt, reads back with ds_read_b128.
template <int G, int AUX>
__global__ __launch_bounds__(256) void lds_read(const float* __restrict__ src, int64_t nvec, uint32_t* out) {
  extern __shared__ f32x4 ring[];  // [4 waves][2][G][64]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  f32x4* my = ring + wave * 2 * G * 64;
  uint32_t x = 0;
  const int64_t per_wave_group = 64 * G;  // vectors
  const int64_t total_waves = (int64_t)gridDim.x * 4;
  const int64_t wid = (int64_t)blockIdx.x * 4 + wave;
  int buf = 0;
  int64_t g0 = wid * per_wave_group;
  const int64_t step = total_waves * per_wave_group;
  auto issue = [&](int64_t gbase, int b) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float GA* p = (const float GA*)(src + (gbase + g * 64 + lane) * 4);
      __builtin_amdgcn_global_load_lds(p, (void LA*)(my + (b * G + g) * 64), 16, 0, AUX);
    }
  };
  if (g0 + per_wave_group <= nvec) issue(g0, 0);
  for (int64_t g = g0; g + per_wave_group <= nvec; g += step) {
    const int64_t nxt = g + step;
    const bool more = nxt + per_wave_group <= nvec;
    if (more) { issue(nxt, buf ^ 1); asm volatile("s_waitcnt vmcnt(%0)" :: "n"(G) : "memory"); }
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < G; ++i) {
      f32x4 v = my[(buf * G + i) * 64 + lane];
      x ^= __float_as_uint(v.x) ^ __float_as_uint(v.y) ^ __float_as_uint(v.z) ^ __float_as_uint(v.w);
    }
    buf ^= 1;
  }
  if (x == 0x12345678u) out[blockIdx.x] = x;
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  f(); f(); hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); return ms / reps;
}

int main() {
  const int64_t bytes = 4ll << 30;
  float* src; uint32_t* out;
  hipMalloc(&src, bytes); hipMalloc(&out, 1 << 20);
  hipMemset(src, 0x3c, bytes);
  const int64_t nvec = bytes / 16;
  auto rep = [&](const char* name, float ms) { printf("%-28s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9); };
  for (int blocks : {2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, 64, "reg G4 b%d", blocks); rep(nm, timeit([&]{ hipLaunchKernelGGL((reg_read<4,false>), dim3(blocks), dim3(256), 0, 0, (const f32x4*)src, nvec, out); }, 10));
    snprintf(nm, 64, "reg G8 b%d", blocks); rep(nm, timeit([&]{ hipLaunchKernelGGL((reg_read<8,false>), dim3(blocks), dim3(256), 0, 0, (const f32x4*)src, nvec, out); }, 10));
    snprintf(nm, 64, "reg G8 nt b%d", blocks); rep(nm, timeit([&]{ hipLaunchKernelGGL((reg_read<8,true>), dim3(blocks), dim3(256), 0, 0, (const f32x4*)src, nvec, out); }, 10));
    snprintf(nm, 64, "reg G16 b%d", blocks); rep(nm, timeit([&]{ hipLaunchKernelGGL((reg_read<16,false>), dim3(blocks), dim3(256), 0, 0, (const f32x4*)src, nvec, out); }, 10));
  }
  for (int blocks : {512, 1024, 2048}) {
    char nm[64];
    snprintf(nm, 64, "lds G4 aux0 b%d", blocks); rep(nm, timeit([&]{ hipLaunchKernelGGL((lds_read<4,0>), dim3(blocks), dim3(256), 4*2*4*64*16, 0, src, nvec, out); }, 10));
    snprintf(nm, 64, "lds G4 aux2 b%d", blocks); rep(nm, timeit([&]{ hipLaunchKernelGGL((lds_read<4,2>), dim3(blocks), dim3(256), 4*2*4*64*16, 0, src, nvec, out); }, 10));
    snprintf(nm, 64, "lds G8 aux2 b%d", blocks); rep(nm, timeit([&]{ hipLaunchKernelGGL((lds_read<8,2>), dim3(blocks), dim3(256), 4*2*8*64*16, 0, src, nvec, out); }, 10));
    snprintf(nm, 64, "lds G8 aux0 b%d", blocks); rep(nm, timeit([&]{ hipLaunchKernelGGL((lds_read<8,0>), dim3(blocks), dim3(256), 4*2*8*64*16, 0, src, nvec, out); }, 10));
  }
  // copy for reference
  return 0;
}
