// Store-pattern microbenchmark for the assembly kernels' output stream: persistent single-wave workgroups,
// each writing whole tiles (one contiguous region of L doubles per tile) with 16-byte buffer stores, as
// swipdg_persistent_kernel does.  Variants: region starts 128-B aligned / 16-B aligned / 8-B aligned
// (head double written separately), tile lengths of P1 (2304 doubles) and Q1 (5120) row-block images,
// workgroups per CU 2..8, optional nontemporal stores, 128-B-aligned instruction footprints.
// Build: hipcc -O3 --offload-arch=gfx950 tilewrite.hip -o tilewrite
#include <hip/hip_runtime.h>
#pragma clang diagnostic ignored "-Wunused-result"
#include <algorithm>
#include <cstdio>
#include <vector>
typedef double dvec2 __attribute__((ext_vector_type(2)));
typedef int ivec4 __attribute__((ext_vector_type(4)));

// tile t covers [t*L + shift, (t+1)*L + shift) doubles (the last one clipped to n)
template <int L, int NT>
__global__ void __launch_bounds__(NT, 1) tw(double* out, long ntiles, int shift, int aux, int align128)
{
  constexpr int STORES = (L / 2 + NT - 1) / NT;
  const long G = gridDim.x, b = blockIdx.x;
  const long x = b & 7, w = b >> 3, gx = G >> 3;
  long t = (ntiles * x) / 8 + w;
  const long t_end = (ntiles * (x + 1)) / 8;
  const int tid = threadIdx.x;
  for (; t < t_end; t += gx) {
    const long base = t * L + shift, tend = base + L;
    const long start = (base + 1) & ~1L, stop = tend & ~1L;
    if (tid == 0) out[base] = 1.0;
    if (tid == 1) out[tend - 1] = 2.0;
    if (!align128) {
      const int nbytes = int(stop - start) * 8;
      __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out + start, (short)0, nbytes, 0x00020000);
#pragma unroll
      for (int k = 0; k < STORES; ++k) {
        const int idx = 2 * (tid + NT * k);
        dvec2 v = {double(idx), double(k)};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), r, idx * 8, aux, 0);
      }
    } else {   // instruction footprints on 128-B lines: chunks outside [start, stop) masked off
      const long a0 = start & ~15L;
      __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out + a0, (short)0, int(stop - a0) * 8, 0x00020000);
#pragma unroll
      for (int k = 0; k < STORES + 1; ++k) {
        const int idx = 2 * (tid + NT * k);
        dvec2 v = {double(idx), double(k)};
        if (a0 + idx >= start) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), r, idx * 8, aux, 0);
      }
    }
  }
}

template <int L, int NT>
static void run(double* out, long n, int cus)
{
  const long ntiles = (n - 64) / L;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int wgcu : {2, 3, 4, 6, 8}) {
    if (long(L) * 8 * wgcu > 160 * 1024 && L > 3000 && wgcu > 3) continue;   // what the real kernel can host
    for (int shift : {0, 2, 1}) {
      for (int mode = 0; mode < 3; ++mode) {
        if (mode == 2 && shift != 2) continue;
        const int aux = mode == 1 ? 2 : 0;   // slc (nontemporal)
        const int al = mode == 2;
        std::vector<float> ts;
        for (int r = 0; r < 9; ++r) {
          hipEventRecord(e0);
          tw<L, NT><<<cus * wgcu, NT>>>(out, ntiles, shift, aux, al);
          hipEventRecord(e1);
          hipEventSynchronize(e1);
          float ms;
          hipEventElapsedTime(&ms, e0, e1);
          ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const double bytes = double(ntiles) * L * 8;
        printf("L=%5d NT=%3d wg/cu=%d shift=%d %-9s median %.4f ms  %6.0f GB/s\n", L, NT, wgcu, shift,
               mode == 0 ? "plain" : (mode == 1 ? "slc" : "align128"), ts[4], bytes / (ts[4] * 1e-3) / 1e9);
      }
    }
  }
}

int main()
{
  const long bytes = 2700L << 20, n = bytes / 8;
  double* out;
  hipMalloc(&out, bytes + 4096);
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  run<2304, 64>(out, n, cus);
  run<5120, 64>(out, n, cus);
  run<5120, 128>(out, n, cus);
  return 0;
}
