// Write-stream microbenchmark: which store organisation reaches the HBM write ceiling on gfx950?
// The C2 kernel's store phase (one 64-lane wave streams an 18 KB tile image with 16-byte non-temporal buffer
// stores, persistent waves, XCD-eighths tile schedule) reaches ~5.9-6.0 TB/s alone, torch's fill_ ~6.5 TB/s.
// Variants over the same 1.18 GB (64000 tiles x 2304 doubles):
//   tile   : the production store phase (persistent, 1 wave per workgroup, WG/CU sweep, XCD eighths) -- nt / plain
//   tileN  : non-persistent, one tile per workgroup
//   fill   : torch-like grid (256 threads, 32 B per thread, non-persistent) -- plain / nt
//   chunk  : persistent 1 KB chunks, grid-stride
//   tile4  : 4-wave workgroups, each wave one of 4 consecutive tiles (adjacent 18 KB streams)
// Build: hipcc -O3 --offload-arch=gfx950 wstream.hip -o wstream
#include <hip/hip_runtime.h>
#pragma clang diagnostic ignored "-Wunused-result"
#include <cstdio>
#include <vector>
typedef double dvec2 __attribute__((ext_vector_type(2)));
typedef int ivec4 __attribute__((ext_vector_type(4)));

constexpr int RB = 36, IMG = 64 * RB, STORES = (IMG / 2 + 63) / 64;

template <int AUX>
__device__ __forceinline__ void store_tile(double* out, long t, const double* lds, int lane)
{
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out + t * IMG, (short)0, IMG * 8, 0x00020000);
#pragma unroll
  for (int k = 0; k < STORES; ++k) {
    const int idx = 2 * (lane + 64 * k);
    const dvec2 v = *reinterpret_cast<const dvec2*>(lds + (idx < IMG ? idx : 0));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), r, idx * 8, 0, AUX);
  }
}

// SCHED 0: XCD eighths; 1: global round robin; 2: XCD-interleaved (tile t on XCD t & 7: adjacent tiles on
// different XCDs, every XCD sweeps the whole range)
template <int AUX, int SCHED>
__global__ void __launch_bounds__(64, 1) tile(double* out, long ntiles)
{
  __shared__ __attribute__((aligned(16))) double lds[IMG];
  const int lane = threadIdx.x;
  const long G = gridDim.x, b = blockIdx.x, x = b & 7, w = b >> 3, gx = G >> 3;
  long t, t_end, step;
  if (SCHED == 0) { t = (ntiles * x) / 8 + w; t_end = (ntiles * (x + 1)) / 8; step = gx; }
  else { t = b; t_end = ntiles; step = G; }
  for (int j = 0; j < RB; ++j) lds[lane * RB + j] = j;
  __builtin_amdgcn_wave_barrier();
  for (; t < t_end; t += step) store_tile<AUX>(out, t, lds, lane);
}

template <int AUX>
__global__ void __launch_bounds__(64, 1) tileN(double* out, long ntiles)
{
  __shared__ __attribute__((aligned(16))) double lds[IMG];
  const int lane = threadIdx.x;
  for (int j = 0; j < RB; ++j) lds[lane * RB + j] = j;
  __builtin_amdgcn_wave_barrier();
  store_tile<AUX>(out, blockIdx.x, lds, lane);
}

template <int AUX>
__global__ void __launch_bounds__(256) tile4(double* out, long ntiles)
{
  __shared__ __attribute__((aligned(16))) double lds[4][IMG];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long G = gridDim.x, b = blockIdx.x, x = b & 7, w = b >> 3, gx = G >> 3;
  const long ng = ntiles / 4;
  long t = (ng * x) / 8 + w, t_end = (ng * (x + 1)) / 8;
  for (int j = 0; j < RB; ++j) lds[wv][lane * RB + j] = j;
  __builtin_amdgcn_wave_barrier();
  for (; t < t_end; t += gx) store_tile<AUX>(out, 4 * t + wv, lds[wv], lane);
}

template <bool NT>
__global__ void __launch_bounds__(256) fill(double* out, long n)
{
  const long i = (long(blockIdx.x) * 256 + threadIdx.x) * 4;
  if (i + 3 < n) {
    const dvec2 v = {1.0, 2.0};
    if (NT) {
      __builtin_nontemporal_store(v, reinterpret_cast<dvec2*>(out + i));
      __builtin_nontemporal_store(v, reinterpret_cast<dvec2*>(out + i + 2));
    } else {
      *reinterpret_cast<dvec2*>(out + i) = v;
      *reinterpret_cast<dvec2*>(out + i + 2) = v;
    }
  }
}

template <bool NT>
__global__ void __launch_bounds__(64) chunk(double* out, long n)
{
  const long G = gridDim.x, nch = n / 128;
  const dvec2 v = {1.0, 2.0};
  for (long c = blockIdx.x; c < nch; c += G) {
    dvec2* p = reinterpret_cast<dvec2*>(out + c * 128 + 2 * threadIdx.x);
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
  }
}

int main()
{
  const long ntiles = 64000, n = ntiles * IMG;
  double* out;
  hipMalloc(&out, n * 8);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const double bytes = double(n) * 8;
  auto time = [&](const char* name, auto launch) {
    launch(); hipDeviceSynchronize();
    float best = 1e9, sum = 0;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      for (int r = 0; r < 20; ++r) launch();
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms = 0; hipEventElapsedTime(&ms, e0, e1); ms /= 20;
      best = ms < best ? ms : best; sum += ms;
    }
    printf("%-36s %8.4f ms (mean %8.4f)  %6.2f TB/s\n", name, best, sum / 3, bytes / (best * 1e-3) / 1e12);
    fflush(stdout);
  };
  char nm[128];
  for (int pass = 0; pass < 2; ++pass) {
    printf("-- pass %d (%.3f GB, %d CUs)\n", pass, bytes / 1e9, cus);
    for (int wg : {2, 4, 8}) {
      snprintf(nm, sizeof nm, "tile nt  eighths wg/cu=%d", wg);
      time(nm, [&] { hipLaunchKernelGGL((tile<2, 0>), dim3(cus * wg), dim3(64), 0, 0, out, ntiles); });
      snprintf(nm, sizeof nm, "tile pl  eighths wg/cu=%d", wg);
      time(nm, [&] { hipLaunchKernelGGL((tile<0, 0>), dim3(cus * wg), dim3(64), 0, 0, out, ntiles); });
      snprintf(nm, sizeof nm, "tile nt  rrobin  wg/cu=%d", wg);
      time(nm, [&] { hipLaunchKernelGGL((tile<2, 1>), dim3(cus * wg), dim3(64), 0, 0, out, ntiles); });
      snprintf(nm, sizeof nm, "tile4 nt eighths wg/cu=%d", wg);
      time(nm, [&] { hipLaunchKernelGGL((tile4<2>), dim3(cus * wg / 4 > 0 ? cus * wg / 4 : cus), dim3(256), 0, 0, out, ntiles); });
    }
    time("tileN nt (one tile per WG)", [&] { hipLaunchKernelGGL((tileN<2>), dim3(ntiles), dim3(64), 0, 0, out, ntiles); });
    time("tileN pl (one tile per WG)", [&] { hipLaunchKernelGGL((tileN<0>), dim3(ntiles), dim3(64), 0, 0, out, ntiles); });
    time("fill plain 256x32B", [&] { hipLaunchKernelGGL((fill<false>), dim3((n / 4 + 255) / 256), dim3(256), 0, 0, out, n); });
    time("fill nt 256x32B", [&] { hipLaunchKernelGGL((fill<true>), dim3((n / 4 + 255) / 256), dim3(256), 0, 0, out, n); });
    for (int wg : {4, 8, 16}) {
      snprintf(nm, sizeof nm, "chunk nt 1KB wg/cu=%d", wg);
      time(nm, [&] { hipLaunchKernelGGL((chunk<true>), dim3(cus * wg), dim3(64), 0, 0, out, n); });
      snprintf(nm, sizeof nm, "chunk pl 1KB wg/cu=%d", wg);
      time(nm, [&] { hipLaunchKernelGGL((chunk<false>), dim3(cus * wg), dim3(64), 0, 0, out, n); });
    }
    time("hipMemsetAsync", [&] { hipMemsetAsync(out, 0, n * 8, 0); });
  }
  return 0;
}
