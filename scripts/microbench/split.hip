// Memory-structure microbenchmark for the C2 kernel (swipdg_persistent_kernel<P1PwcPolicy>): the same
// per-tile traffic -- 64 elements per tile, 9 own doubles + 3 neighbour ids per element (SoA, coalesced),
// 3 gathered doubles per face from the neighbour, a 2304-double (18 KB) row-block image streamed out with
// 16-byte non-temporal buffer stores -- under two wave organisations:
//   mono : one wave per workgroup loads, computes and stores (the production kernel's order
//          [own t+1][compute t][gathers t+1][stores t]); gfx950's vmcnt is in order and counts stores, so
//          the gathers of t+1 wait for the stores of t-1;
//   split: two waves per workgroup, a loader wave (own + gathers, 3 tiles of own data and 1 tile of
//          gathers in flight, staged into a 2-slot LDS ring) and a compute/store wave that never loads from
//          global memory, so none of its waits covers a store; one s_barrier per tile.
// `work` adds dependent f64 FMAs per lane per tile to emulate the closed-form compute.
// Build: hipcc -O3 --offload-arch=gfx950 split.hip -o split
#include <hip/hip_runtime.h>
#pragma clang diagnostic ignored "-Wunused-result"
#include <algorithm>
#include <cstdio>
#include <type_traits>
#include <vector>
typedef double dvec2 __attribute__((ext_vector_type(2)));
typedef int ivec4 __attribute__((ext_vector_type(4)));

constexpr int RB = 36, IMG = 64 * RB, STORES = (IMG / 2 + 63) / 64, NO = 9, NG = 9;

struct Args {
  const double* own;   // [NO][n]
  const int* nbr;      // [3][n]
  double* out;         // [ntiles * IMG]
  long n, ntiles;
  int work;
};

struct Own { double v[NO]; int nb[3]; };
struct Gat { double g[NG]; };

__device__ __forceinline__ void load_own(const Args& a, long e, Own& o)
{
#pragma unroll
  for (int k = 0; k < NO; ++k) o.v[k] = a.own[k * a.n + e];
#pragma unroll
  for (int f = 0; f < 3; ++f) o.nb[f] = a.nbr[f * a.n + e];
}
__device__ __forceinline__ void load_gat(const Args& a, long e, const Own& o, Gat& g)
{
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    const long m = o.nb[f] >= 0 ? long(o.nb[f]) : e;
#pragma unroll
    for (int k = 0; k < 3; ++k) g.g[3 * f + k] = a.own[k * a.n + m];
  }
}
__device__ __forceinline__ void compute(const Args& a, const double* ov, const double* gv, double* img)
{
  double acc[NO];
#pragma unroll
  for (int k = 0; k < NO; ++k) acc[k] = ov[k] * gv[k];
  for (int w = 0; w < a.work; ++w)
#pragma unroll
    for (int k = 0; k < NO; ++k) acc[k] = fma(acc[k], 0.999, gv[k]);
#pragma unroll
  for (int j = 0; j < RB; ++j) img[j] = acc[j % NO] + double(j);
}

__device__ int g_sched;   // 0: XCD eighths (production); 1: global round robin; 2: per-window XCD slices
__device__ __forceinline__ void sched(long ntiles, long& t, long& t_end, long& step)
{
  const long G = gridDim.x, b = blockIdx.x, x = b & 7, w = b >> 3, gx = G >> 3;
  if (g_sched == 1) {
    t = b; t_end = ntiles; step = G;
  } else if (g_sched == 2) {   // window k = tiles [k G, (k+1) G); XCD x takes slice [x G/8, (x+1) G/8) of it
    t = x * gx + w; t_end = ntiles; step = G;
  } else {
    t = (ntiles * x) / 8 + w;
    t_end = (ntiles * (x + 1)) / 8;
    step = gx;
  }
}

template <int AUX>
__device__ __forceinline__ void store_tile(const Args& a, long t, const double* lds, int lane)
{
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(a.out + t * IMG, (short)0, IMG * 8, 0x00020000);
#pragma unroll
  for (int k = 0; k < STORES; ++k) {
    const int idx = 2 * (lane + 64 * k);
    const dvec2 v = *reinterpret_cast<const dvec2*>(lds + (idx < IMG ? idx : 0));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), r, idx * 8, 0, AUX);
  }
}

template <int AUX>
__global__ void __launch_bounds__(64, 1) mono(const Args a)
{
  __shared__ __attribute__((aligned(16))) double lds[IMG];
  const int lane = threadIdx.x;
  long t, t_end, step;
  sched(a.ntiles, t, t_end, step);
  if (t >= t_end) return;
  Own own; Gat gat;
  load_own(a, t * 64 + lane, own);
  load_gat(a, t * 64 + lane, own, gat);
  for (;;) {
    const bool has_next = t + step < t_end;
    const long tn = has_next ? t + step : t;
    Own own_n;
    load_own(a, tn * 64 + lane, own_n);
    compute(a, own.v, gat.g, lds + lane * RB);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    Gat gat_n;
    load_gat(a, tn * 64 + lane, own_n, gat_n);
    store_tile<AUX>(a, t, lds, lane);
    if (!has_next) break;
    t = tn; own = own_n; gat = gat_n;
  }
}

// LDS-only wait + workgroup barrier: the waits the compiler would emit for __syncthreads() include
// vmcnt(0), i.e. the compute wave's outstanding stores
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int AUX>
__global__ void __launch_bounds__(128, 1) split(const Args a)
{
  __shared__ __attribute__((aligned(16))) double img[IMG];
  __shared__ double ring[2][NO + NG][64];
  const int lane = threadIdx.x & 63;
  const bool loader = threadIdx.x < 64;
  long t0, t_end, step;
  sched(a.ntiles, t0, t_end, step);
  if (t0 >= t_end) return;
  const long nt = (t_end - t0 + step - 1) / step;
  auto tile = [&](long i) { return t0 + (i < nt ? i : nt - 1) * step; };
  if (loader) {
    Own o0, o1, o2;
    Gat g;
    load_own(a, tile(0) * 64 + lane, o0);
    load_own(a, tile(1) * 64 + lane, o1);
    load_gat(a, tile(0) * 64 + lane, o0, g);
    load_own(a, tile(2) * 64 + lane, o2);
    for (long i = 0; i < nt; ++i) {
      double* s = &ring[i & 1][0][0];
#pragma unroll
      for (int k = 0; k < NO; ++k) s[k * 64 + lane] = o0.v[k];
#pragma unroll
      for (int k = 0; k < NG; ++k) s[(NO + k) * 64 + lane] = g.g[k];
      lds_barrier();
      load_gat(a, tile(i + 1) * 64 + lane, o1, g);
      o0 = o1; o1 = o2;
      load_own(a, tile(i + 3) * 64 + lane, o2);
    }
  } else {
    for (long i = 0; i < nt; ++i) {
      lds_barrier();
      double ov[NO], gv[NG];
      const double* s = &ring[i & 1][0][0];
#pragma unroll
      for (int k = 0; k < NO; ++k) ov[k] = s[k * 64 + lane];
#pragma unroll
      for (int k = 0; k < NG; ++k) gv[k] = s[(NO + k) * 64 + lane];
      compute(a, ov, gv, img + lane * RB);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      store_tile<AUX>(a, tile(i), img, lane);
    }
  }
}

template <int AUX>
__global__ void fillchunks(const Args a)
{
  const int lane = threadIdx.x;
  const long G = gridDim.x, nchunks = a.ntiles * IMG / 128;   // 1 KB = 128 doubles per wave instruction
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(a.out, (short)0, 0x7fffffff, 0x00020000);
  for (long c = blockIdx.x; c < nchunks; c += G) {
    const dvec2 v = {double(c), 1.0};
    const long off = (c * 128 + 2 * lane) * 8;
    double* p = a.out + c * 128 + 2 * lane;
    __builtin_nontemporal_store(v, reinterpret_cast<dvec2*>(p));
    (void)off; (void)r;
  }
}

template <int AUX>
__global__ void storeonly(const Args a)
{
  __shared__ __attribute__((aligned(16))) double lds[IMG];
  const int lane = threadIdx.x;
  long t, t_end, step;
  sched(a.ntiles, t, t_end, step);
  for (int j = 0; j < RB; ++j) lds[lane * RB + j] = j;
  __builtin_amdgcn_wave_barrier();
  for (; t < t_end; t += step) store_tile<AUX>(a, t, lds, lane);
}

int main()
{
  const long n = 4096000, ntiles = n / 64;
  Args a{};
  a.n = n; a.ntiles = ntiles;
  std::vector<double> h(NO * n);
  for (long i = 0; i < NO * n; ++i) h[i] = 1.0 + 1e-9 * double(i % 1000);
  std::vector<int> nb(3 * n);
  const long ny = 1280;   // neighbours like a Kuhn strip: e-1, e+1, e +- column
  for (long e = 0; e < n; ++e) {
    nb[e] = e > 0 ? int(e - 1) : -1;
    nb[n + e] = e + 1 < n ? int(e + 1) : -1;
    const long c = (e & 1) ? e + ny - 1 : e - ny + 1;
    nb[2 * n + e] = (c >= 0 && c < n) ? int(c) : -1;
  }
  double *own, *out; int* nbr;
  hipMalloc(&own, NO * n * 8); hipMalloc(&nbr, 3 * n * 4); hipMalloc(&out, ntiles * IMG * 8);
  hipMemcpy(own, h.data(), NO * n * 8, hipMemcpyHostToDevice);
  hipMemcpy(nbr, nb.data(), 3 * n * 4, hipMemcpyHostToDevice);
  a.own = own; a.nbr = nbr; a.out = out;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const double bytes = double(ntiles) * IMG * 8 + double(n) * (NO * 8 + 12);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  auto time = [&](const char* name, auto launch) {
    launch(); hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 20; ++r) launch();
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms = 0; hipEventElapsedTime(&ms, e0, e1); ms /= 20;
    printf("%-34s %8.4f ms  %6.2f TB/s (own+img bytes)\n", name, ms, bytes / (ms * 1e-3) / 1e12);
    fflush(stdout);
  };
  char nm[128];
  for (int sc : {0, 1, 2}) {
    hipMemcpyToSymbol(HIP_SYMBOL(g_sched), &sc, sizeof(int));
    for (int wg : {4, 8}) {
      snprintf(nm, sizeof nm, "storeonly sched=%d wg/cu=%d", sc, wg);
      time(nm, [&] { hipLaunchKernelGGL(storeonly<2>, dim3(cus * wg), dim3(64), 0, 0, a); });
      snprintf(nm, sizeof nm, "mono      sched=%d wg/cu=%d", sc, wg);
      time(nm, [&] { hipLaunchKernelGGL(mono<2>, dim3(cus * wg), dim3(64), 0, 0, a); });
    }
  }
  for (int wg : {4, 8, 16}) {
    snprintf(nm, sizeof nm, "fillchunks 1KB nt wg/cu=%d", wg);
    time(nm, [&] { hipLaunchKernelGGL(fillchunks<2>, dim3(cus * wg), dim3(64), 0, 0, a); });
  }
  // correctness of the split image: tile 5, element 3, value 7
  std::vector<double> o(IMG);
  hipMemcpy(o.data(), out + 5 * IMG, IMG * 8, hipMemcpyDeviceToHost);
  printf("check %.6f %.6f\n", o[3 * RB + 7], o[60 * RB + 35]);
  return 0;
}
