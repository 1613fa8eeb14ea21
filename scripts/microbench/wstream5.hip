// Write-stream microbenchmark, part 5 (chunk size per wave; after wstream.hip: torch-like fill 6.7 TB/s, the C2 tile store phase
// 5.8-6.1 TB/s).  Separates the factors: bytes per lane per chunk (16 / 32 / 64 B, adjacent stores of one
// lane = "lane-contiguous", or one 1 KB wave instruction after another = "instr-contiguous"), workgroup size
// (64 / 256), persistent grid-stride vs one chunk per workgroup, store policy (plain / nt), and the C2 tile
// (18 KB per wave) written lane-contiguous.
// Build: hipcc -O3 --offload-arch=gfx950 -Wno-unused-result wstream2.hip -o wstream2
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dvec2 __attribute__((ext_vector_type(2)));
typedef int ivec4 __attribute__((ext_vector_type(4)));

constexpr int RB = 36, IMG = 64 * RB;

template <bool NT>
__device__ __forceinline__ void st(double* p, dvec2 v)
{
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<dvec2*>(p));
  else *reinterpret_cast<dvec2*>(p) = v;
}

// one chunk = WG threads x K stores of 16 B; LC: lane-contiguous (thread i writes [16 K i, 16 K (i+1))),
// else instruction-contiguous (store k of the wave covers 1 KB at k KB)
template <int K, bool LC, bool NT>
__device__ __forceinline__ void chunk_store(double* base, int tid, int nthr)
{
  const dvec2 v = {1.0, 2.0};
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const long off = LC ? (long(tid) * K + k) * 2 : (long(k) * nthr + tid) * 2;
    st<NT>(base + off, v);
  }
}

template <int K, bool LC, bool NT, int WG>
__global__ void __launch_bounds__(WG) fillN(double* out, long n)
{
  const long per = long(WG) * K * 2;
  const long c = blockIdx.x;
  if ((c + 1) * per <= n) chunk_store<K, LC, NT>(out + c * per, threadIdx.x, WG);
}

template <int K, bool LC, bool NT, int WG>
__global__ void __launch_bounds__(WG) fillP(double* out, long n)
{
  const long per = long(WG) * K * 2, nch = n / per;
  for (long c = blockIdx.x; c < nch; c += gridDim.x) chunk_store<K, LC, NT>(out + c * per, threadIdx.x, WG);
}

// persistent fill, XCD eighths (each XCD sweeps a contiguous eighth of the chunks)
template <int K, bool LC, bool NT, int WG>
__global__ void __launch_bounds__(WG) fillE(double* out, long n)
{
  const long per = long(WG) * K * 2, nch = n / per;
  const long G = gridDim.x, b = blockIdx.x, x = b & 7, w = b >> 3, gx = G >> 3;
  for (long c = (nch * x) / 8 + w; c < (nch * (x + 1)) / 8; c += gx)
    chunk_store<K, LC, NT>(out + c * per, threadIdx.x, WG);
}

// the C2 tile (2304 doubles = 18 KB) from an LDS image, 1 wave, persistent XCD eighths, lane-contiguous
// pairs: lane l writes 32 B at [32 l, 32 l + 32) of each 2 KB span (9 spans per tile)
template <bool NT, bool LC>
__global__ void __launch_bounds__(64, 1) tileS(double* out, long ntiles)
{
  __shared__ __attribute__((aligned(16))) double lds[IMG];
  const int lane = threadIdx.x;
  const long G = gridDim.x, b = blockIdx.x, x = b & 7, w = b >> 3, gx = G >> 3;
  for (int j = 0; j < RB; ++j) lds[lane * RB + j] = j;
  __builtin_amdgcn_wave_barrier();
  for (long t = (ntiles * x) / 8 + w; t < (ntiles * (x + 1)) / 8; t += gx) {
    double* o = out + t * IMG;
#pragma unroll
    for (int s = 0; s < IMG / 256; ++s) {   // 9 spans of 256 doubles
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int idx = LC ? s * 256 + 4 * lane + 2 * h : s * 256 + 128 * h + 2 * lane;
        const dvec2 v = *reinterpret_cast<const dvec2*>(lds + idx);
        st<NT>(o + idx, v);
      }
    }
  }
}

int main()
{
  const long ntiles = 64000, n = ntiles * IMG;
  double* out;
  (void)hipMalloc(&out, n * 8);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  const double bytes = double(n) * 8;
  auto time = [&](const char* name, auto launch) {
    launch(); (void)hipDeviceSynchronize();
    float best = 1e9;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0);
      for (int r = 0; r < 20; ++r) launch();
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1); ms /= 20;
      best = ms < best ? ms : best;
    }
    printf("%-40s %8.4f ms  %6.2f TB/s\n", name, best, bytes / (best * 1e-3) / 1e12);
    fflush(stdout);
  };
#define PERS(KIND, K, LC, NT, WG, M) \
  time(#KIND " K=" #K " LC=" #LC " NT=" #NT " WG=" #WG " x" #M, [&] { \
    hipLaunchKernelGGL((KIND<K, LC, NT, WG>), dim3(cus * M), dim3(WG), 0, 0, out, n); })
  for (int pass = 0; pass < 2; ++pass) {
    printf("-- pass %d: per-wave chunk size (K KB per iteration), XCD eighths, 64-lane waves\n", pass);
    PERS(fillE, 1, false, true, 64, 4); PERS(fillE, 2, false, true, 64, 4); PERS(fillE, 4, false, true, 64, 4);
    PERS(fillE, 9, false, true, 64, 4); PERS(fillE, 18, false, true, 64, 4); PERS(fillE, 36, false, true, 64, 4);
    PERS(fillE, 2, false, true, 64, 8); PERS(fillE, 9, false, true, 64, 8); PERS(fillE, 18, false, true, 64, 8);
    PERS(fillE, 9, false, true, 64, 2); PERS(fillE, 18, false, true, 64, 2);
    PERS(fillE, 1, false, false, 64, 4); PERS(fillE, 2, false, false, 64, 4); PERS(fillE, 9, false, false, 64, 4);
    PERS(fillE, 2, true, true, 64, 4); PERS(fillE, 2, true, false, 64, 4);
  }
  return 0;
}
