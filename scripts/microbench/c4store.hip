// C4 store-organisation microbenchmark: store-only, the exact CSR value array of the C4 workload
// (SPE10 3520 x 1200 Q1, 8 x 8 subdomains, subdomain-major element order, AllDirichlet: 337,768,960 values =
// 2.70 GB), written in CSR order by tiles of 64 consecutive elements, under the organisations a kernel could use:
//
//   half20   per-wave 20 KB half images (32 row blocks), 2 waves per SIMD: today's Q1 kernel (swipdg_device.hh HALF)
//   whole40  per-wave 40 KB whole-tile images, 1 wave per SIMD (round-1..3 Q1 kernel)
//   coopW_T  a workgroup of W waves owns T adjacent tiles (T x 40 KB image); after a barrier all W waves stream the
//            joint CSR range in 1 KB chunks interleaved over the waves (store k of thread i at 16 (i + 64 W k))
//   fill4k   torch-like fill of the same bytes (256-thread workgroups, one 4 KB chunk each, not persistent)
//   fillE1k  persistent XCD-eighths fill, each wave 1 KB per iteration (the densest persistent write front)
//
// Every persistent variant sweeps XCD eighths of its unit range as the production kernels do (blockIdx & 7 = XCD).
// The image is read back from LDS with ds_read_b128 (as the kernels do) and stored with non-temporal 16-byte
// buffer stores whose descriptor range drops the tail.  LDS writes of the image (40 ds_write_b64 per lane per 20 KB)
// are issued as in the kernel, without compute.  Output: best / median of 3 x 20 back-to-back launches, TB/s.
// Build: hipcc -O3 --offload-arch=gfx950 c4store.hip -o c4store
#include <hip/hip_runtime.h>
#pragma clang diagnostic ignored "-Wunused-result"
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>
typedef double dvec2 __attribute__((ext_vector_type(2)));
typedef int ivec4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st16(const dvec2& v, __amdgpu_buffer_rsrc_t r, int off)
{
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), r, off, 0, 2);   // nt
}
__device__ __forceinline__ void lds_sync()
{
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// XCD-eighths sweep of n units by G workgroups: unit sequence of workgroup b
struct Sweep {
  int64_t u, end, step;
  __device__ Sweep(int64_t n)
  {
    const int64_t G = gridDim.x, b = blockIdx.x, x = b & 7, w = b >> 3, gx = G >> 3;
    u = (n * x) / 8 + w;
    end = (n * (x + 1)) / 8;
    step = gx;
  }
};
// XCD-interleaved sweep: XCD x owns the units u with (u / K) % 8 == x (K = 1: global round robin); its waves take
// its j-th unit for j = w, w + gx, ... (gSweep::next returns -1 when done)
struct gSweep {
  int64_t j, step, n, K, x;
  __device__ gSweep(int64_t n_, int64_t K_) : n(n_), K(K_)
  {
    const int64_t G = gridDim.x, b = blockIdx.x;
    x = b & 7;
    j = b >> 3;
    step = G >> 3;
  }
  __device__ int64_t unit() const { return (j / K) * 8 * K + x * K + j % K; }
};

// per-wave images of NBLK row blocks (32: half images, 64: whole tiles), one wave per workgroup
template <int NBLK>
__global__ void __launch_bounds__(64) waveimg(double* out, const int64_t* __restrict__ ptr, int64_t ntiles)
{
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int IMG = NBLK * 80, ST = IMG / 128;   // doubles per image, 1 KB stores per image
  const int lane = threadIdx.x;
  char* ldsb = reinterpret_cast<char*>(lds);
  for (Sweep s(ntiles); s.u < s.end; s.u += s.step) {
    const int64_t e0 = s.u * 64;
#pragma unroll
    for (int h = 0; h < 64 / NBLK; ++h) {
      const int64_t b0 = __builtin_amdgcn_readfirstlane(ptr[e0 + NBLK * h]);
      const int64_t b1 = __builtin_amdgcn_readfirstlane(ptr[e0 + NBLK * (h + 1)]);
      // the image: 40 ds_write_b64 per lane per 32 row blocks (values of lane-owned rows)
#pragma unroll
      for (int j = 0; j < IMG / 64; ++j) lds[lane + 64 * j] = double(j + h);
      lds_sync();
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out + b0, (short)0, int(b1 - b0) * 8, 0x00020000);
#pragma unroll
      for (int k = 0; k < ST; ++k) {
        const dvec2 v = *reinterpret_cast<const dvec2*>(ldsb + 16 * lane + 1024 * k);
        st16(v, r, 16 * lane + 1024 * k);
      }
    }
  }
}

// Q1 vertex-indexed own data of one element (what the kernel's load_own / first gather stage read): 4 vertex ids,
// 4 neighbour ids, face info, the per-element tensor (44 B, SoA rows of n), then the 4 vertex rows (16 B each) the ids
// name
struct Mesh {
  const int* ev;      // [4][n]
  const int* nbr;     // [4][n]
  const unsigned* fi; // [n]
  const double* ten;  // [n]
  const double* vx;   // [nv][2]
  int64_t n;
};
struct Own {
  int v[4], nb[4];
  unsigned f;
  double t;
};
__device__ __forceinline__ void load_own(const Mesh& m, int64_t e, Own& o)
{
#pragma unroll
  for (int i = 0; i < 4; ++i) o.v[i] = m.ev[i * m.n + e];
#pragma unroll
  for (int i = 0; i < 4; ++i) o.nb[i] = m.nbr[i * m.n + e];
  o.f = m.fi[e];
  o.t = m.ten[e];
}
__device__ __forceinline__ double use_own(const Mesh& m, const Own& o)
{
  double s = o.t + double(o.f);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const dvec2 c = *reinterpret_cast<const dvec2*>(m.vx + 2 * int64_t(o.v[i]));
    s += c.x + c.y + double(o.nb[i]);
  }
  return s;
}

// waveimg + the own-data stream: tile t+1's records loaded before tile t's stores (in-order vmcnt: the next
// iteration's use waits behind them, as in the kernel), the vertex rows gathered at the top of the next iteration
template <int NBLK>
__global__ void __launch_bounds__(64) waveimgL(double* out, const int64_t* __restrict__ ptr, int64_t ntiles, Mesh m)
{
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int IMG = NBLK * 80, ST = IMG / 128;
  const int lane = threadIdx.x;
  char* ldsb = reinterpret_cast<char*>(lds);
  Sweep s(ntiles);
  if (s.u >= s.end) return;
  Own own, own_n;
  load_own(m, s.u * 64 + lane, own);
  for (; s.u < s.end; s.u += s.step) {
    const int64_t e0 = s.u * 64;
    const int64_t un = s.u + s.step < s.end ? s.u + s.step : s.u;
    const double val = use_own(m, own);
    load_own(m, un * 64 + lane, own_n);
#pragma unroll
    for (int h = 0; h < 64 / NBLK; ++h) {
      const int64_t b0 = __builtin_amdgcn_readfirstlane(ptr[e0 + NBLK * h]);
      const int64_t b1 = __builtin_amdgcn_readfirstlane(ptr[e0 + NBLK * (h + 1)]);
#pragma unroll
      for (int j = 0; j < IMG / 64; ++j) lds[lane + 64 * j] = val + double(j + h);
      lds_sync();
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out + b0, (short)0, int(b1 - b0) * 8, 0x00020000);
#pragma unroll
      for (int k = 0; k < ST; ++k) {
        const dvec2 v = *reinterpret_cast<const dvec2*>(ldsb + 16 * lane + 1024 * k);
        st16(v, r, 16 * lane + 1024 * k);
      }
    }
    own = own_n;
  }
}

// Model of a Q1 kernel with compute: a workgroup of W waves owns a unit of 64 W consecutive elements, one element per
// lane, written in two phases of 32 W elements each (lanes 0-31 of wave w hold element 32 w + l, lanes 32-63 element
// 32 W + 32 w + l - 32), each phase's CSR range (W x 20 KB) staged in LDS and streamed by all W waves in 1 KB chunks
// interleaved over the waves.  W = 1 is today's half-image kernel.  Per lane: the own record of the next unit loaded
// before this unit's stores, NC dependent f64 FMAs (4 chains) standing in for the closed forms, 40 values per phase
// written to LDS (phase 0 right after the compute, phase 1 from registers after phase 0's stores were issued).
// STORE = false: the same without the value stores (what the compute + loads cost alone).
template <int W, int NC, bool STORE>
__global__ void __launch_bounds__(64 * W) coopC(double* out, const int64_t* __restrict__ ptr, int64_t ntiles, Mesh m)
{
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int NTH = 64 * W, PH = 32 * W * 80, ST = PH / 2 / NTH;   // doubles per phase, 16-B stores per thread
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int eo = l < 32 ? 32 * w + l : 32 * W + 32 * w + (l - 32);   // the lane's element in the unit
  char* ldsb = reinterpret_cast<char*>(lds);
  Sweep s(ntiles / W);
  if (s.u >= s.end) return;
  Own own, own_n;
  load_own(m, s.u * NTH + eo, own);
  for (; s.u < s.end; s.u += s.step) {
    const int64_t e0 = s.u * NTH;
    const int64_t un = s.u + s.step < s.end ? s.u + s.step : s.u;
    const double v = use_own(m, own);
    load_own(m, un * NTH + eo, own_n);
    double x[4] = {v, v + 1.0, v + 2.0, v + 3.0};
#pragma unroll 8
    for (int i = 0; i < NC / 4; ++i)
#pragma unroll
      for (int c = 0; c < 4; ++c) x[c] = __builtin_fma(x[c], 0.999999, 1e-7 * c);
    double hold[40];
#pragma unroll
    for (int j = 0; j < 40; ++j) hold[j] = x[j & 3] + double(j);
    __syncthreads();   // the previous unit's phase-1 LDS reads are done
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      // the lane's 40 values of this phase: lanes 0-31 / 32-63 hold rows (0, 1) / (2, 3) of the phase's element l & 31
      // of wave w (after the permlane32 regroup of the real kernel): LDS slot (32 w + (l & 31)) * 80 + 40 (l >> 5) + j
      const int slot = (32 * w + (l & 31)) * 80 + 40 * (l >> 5);
#pragma unroll
      for (int j = 0; j < 40; ++j) lds[slot + j] = hold[j] + double(ph);
      __syncthreads();
      const int64_t b0 = __builtin_amdgcn_readfirstlane(ptr[e0 + 32 * W * ph]);
      const int64_t b1 = __builtin_amdgcn_readfirstlane(ptr[e0 + 32 * W * (ph + 1)]);
      const __amdgpu_buffer_rsrc_t r =
          __builtin_amdgcn_make_buffer_rsrc(out + b0, (short)0, STORE ? int(b1 - b0) * 8 : 0, 0x00020000);
#pragma unroll
      for (int k = 0; k < ST; ++k) {
        const int o = 16 * tid + 16 * NTH * k;
        const dvec2 vv = *reinterpret_cast<const dvec2*>(ldsb + o);
        st16(vv, r, o);
      }
      if (ph == 0) __syncthreads();   // phase 0's LDS reads done before phase 1 overwrites the image
    }
    own = own_n;
  }
}

// coop + the own-data stream (threads < 64 T load one element each)
template <int W, int T>
__global__ void __launch_bounds__(64 * W) coopL(double* out, const int64_t* __restrict__ ptr, int64_t ntiles, Mesh m)
{
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int IMG = T * 64 * 80, NTH = 64 * W, ST = (IMG / 2 + NTH - 1) / NTH;
  const int tid = threadIdx.x;
  const int tl = tid < 64 * T ? tid : 0;
  char* ldsb = reinterpret_cast<char*>(lds);
  Sweep s(ntiles / T);
  if (s.u >= s.end) return;
  Own own, own_n;
  load_own(m, s.u * 64 * T + tl, own);
  for (; s.u < s.end; s.u += s.step) {
    const int64_t e0 = s.u * 64 * T;
    const int64_t un = s.u + s.step < s.end ? s.u + s.step : s.u;
    const double val = use_own(m, own);
    load_own(m, un * 64 * T + tl, own_n);
    const int64_t b0 = __builtin_amdgcn_readfirstlane(ptr[e0]);
    const int64_t b1 = __builtin_amdgcn_readfirstlane(ptr[e0 + 64 * T]);
#pragma unroll
    for (int j = 0; j < IMG / NTH; ++j) lds[tid + NTH * j] = val + double(j);
    __syncthreads();
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out + b0, (short)0, int(b1 - b0) * 8, 0x00020000);
#pragma unroll
    for (int k = 0; k < ST; ++k) {
      const int o = 16 * tid + 16 * NTH * k;
      const dvec2 v = *reinterpret_cast<const dvec2*>(ldsb + (o < IMG * 8 ? o : 0));
      st16(v, r, o);
    }
    __syncthreads();
    own = own_n;
  }
}

// waveimg with the XCD-interleaved sweep (K tiles per XCD chunk); K = 0: one tile per workgroup (not persistent)
template <int NBLK>
__global__ void __launch_bounds__(64) waveimgK(double* out, const int64_t* __restrict__ ptr, int64_t ntiles, int64_t K)
{
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int IMG = NBLK * 80, ST = IMG / 128;
  const int lane = threadIdx.x;
  char* ldsb = reinterpret_cast<char*>(lds);
  gSweep s(ntiles, K > 0 ? K : 1);
  for (;; s.j += s.step) {
    const int64_t u = K > 0 ? s.unit() : int64_t(blockIdx.x);
    if (u >= ntiles) break;
    const int64_t e0 = u * 64;
#pragma unroll
    for (int h = 0; h < 64 / NBLK; ++h) {
      const int64_t b0 = __builtin_amdgcn_readfirstlane(ptr[e0 + NBLK * h]);
      const int64_t b1 = __builtin_amdgcn_readfirstlane(ptr[e0 + NBLK * (h + 1)]);
#pragma unroll
      for (int j = 0; j < IMG / 64; ++j) lds[lane + 64 * j] = double(j + h);
      lds_sync();
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out + b0, (short)0, int(b1 - b0) * 8, 0x00020000);
#pragma unroll
      for (int k = 0; k < ST; ++k) {
        const dvec2 v = *reinterpret_cast<const dvec2*>(ldsb + 16 * lane + 1024 * k);
        st16(v, r, 16 * lane + 1024 * k);
      }
    }
    if (K == 0) break;
  }
}

// workgroup-cooperative: W waves, T tiles per unit, the joint range streamed in 1 KB chunks interleaved over waves
template <int W, int T>
__global__ void __launch_bounds__(64 * W) coop(double* out, const int64_t* __restrict__ ptr, int64_t ntiles)
{
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int IMG = T * 64 * 80, NTH = 64 * W, ST = (IMG / 2 + NTH - 1) / NTH;
  const int tid = threadIdx.x;
  char* ldsb = reinterpret_cast<char*>(lds);
  for (Sweep s(ntiles / T); s.u < s.end; s.u += s.step) {
    const int64_t e0 = s.u * 64 * T;
    const int64_t b0 = __builtin_amdgcn_readfirstlane(ptr[e0]);
    const int64_t b1 = __builtin_amdgcn_readfirstlane(ptr[e0 + 64 * T]);
#pragma unroll
    for (int j = 0; j < IMG / NTH; ++j) lds[tid + NTH * j] = double(j);
    __syncthreads();
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out + b0, (short)0, int(b1 - b0) * 8, 0x00020000);
#pragma unroll
    for (int k = 0; k < ST; ++k) {
      const int o = 16 * tid + 16 * NTH * k;
      const dvec2 v = *reinterpret_cast<const dvec2*>(ldsb + (o < IMG * 8 ? o : 0));
      st16(v, r, o);
    }
    __syncthreads();
  }
}

// not persistent, one tile (two half images) per 64-thread workgroup, the tile index remapped to XCD eighths (workgroup b
// runs on XCD b & 7 and takes tile (b & 7) n / 8 + (b >> 3)), optionally with the own-data loads of its tile
template <int NBLK, bool LOADS>
__global__ void __launch_bounds__(64) waveimgNP(double* out, const int64_t* __restrict__ ptr, int64_t ntiles, Mesh m)
{
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int IMG = NBLK * 80, ST = IMG / 128;
  const int lane = threadIdx.x;
  char* ldsb = reinterpret_cast<char*>(lds);
  const int64_t per = (ntiles + 7) / 8, u = int64_t(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (u >= ntiles || (blockIdx.x >> 3) >= per) return;
  const int64_t e0 = u * 64;
  double val = 0.0;
  if (LOADS) {
    Own own;
    load_own(m, e0 + lane, own);
    val = use_own(m, own);
  }
#pragma unroll
  for (int h = 0; h < 64 / NBLK; ++h) {
    const int64_t b0 = __builtin_amdgcn_readfirstlane(ptr[e0 + NBLK * h]);
    const int64_t b1 = __builtin_amdgcn_readfirstlane(ptr[e0 + NBLK * (h + 1)]);
#pragma unroll
    for (int j = 0; j < IMG / 64; ++j) lds[lane + 64 * j] = val + double(j + h);
    lds_sync();
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out + b0, (short)0, int(b1 - b0) * 8, 0x00020000);
#pragma unroll
    for (int k = 0; k < ST; ++k) {
      const dvec2 v = *reinterpret_cast<const dvec2*>(ldsb + 16 * lane + 1024 * k);
      st16(v, r, 16 * lane + 1024 * k);
    }
  }
}

// torch-like fill with the chunk index remapped to XCD eighths
__global__ void __launch_bounds__(256) fill4kE(double* out, int64_t n)
{
  const int64_t nch = n / 512, per = (nch + 7) / 8, c = int64_t(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  const dvec2 v = {1.0, 2.0};
  if (c < nch && (blockIdx.x >> 3) < per)
    __builtin_nontemporal_store(v, reinterpret_cast<dvec2*>(out + c * 512 + 2 * threadIdx.x));
}

// torch-like fill: one 4 KB chunk per 256-thread workgroup
template <bool NT>
__global__ void __launch_bounds__(256) fill4k(double* out, int64_t n)
{
  const int64_t i = (int64_t(blockIdx.x) * 256 + threadIdx.x) * 2;
  const dvec2 v = {1.0, 2.0};
  if (i + 1 < n) {
    if (NT) __builtin_nontemporal_store(v, reinterpret_cast<dvec2*>(out + i));
    else *reinterpret_cast<dvec2*>(out + i) = v;
  }
}

// persistent fill, XCD-interleaved by chunks of K KB, 1 KB per wave per iteration
__global__ void __launch_bounds__(64) fillK1k(double* out, int64_t n, int64_t K)
{
  const dvec2 v = {1.0, 2.0};
  for (gSweep s(n / 128, K);; s.j += s.step) {
    const int64_t u = s.unit();
    if (u >= n / 128) break;
    __builtin_nontemporal_store(v, reinterpret_cast<dvec2*>(out + u * 128 + 2 * threadIdx.x));
  }
}

// persistent XCD-eighths fill, 1 KB per wave per iteration
__global__ void __launch_bounds__(64) fillE1k(double* out, int64_t n)
{
  const dvec2 v = {1.0, 2.0};
  for (Sweep s(n / 128); s.u < s.end; s.u += s.step)
    __builtin_nontemporal_store(v, reinterpret_cast<dvec2*>(out + s.u * 128 + 2 * threadIdx.x));
}

int main(int argc, char** argv)
{
  const int nx = 3520, ny = 1200, px = 8, py = 8;
  const int passes = argc > 1 ? atoi(argv[1]) : 2;
  // C4 elem_ptr: subdomain-major (s = sx * py + sy), x fastest inside a subdomain, row block 16 (1 + interior faces)
  const int64_t ne = int64_t(nx) * ny;
  std::vector<int64_t> ptr(ne + 1, 0);
  int64_t g = 0;
  for (int sx = 0; sx < px; ++sx)
    for (int sy = 0; sy < py; ++sy) {
      const int i0 = sx * nx / px, i1 = (sx + 1) * nx / px, j0 = sy * ny / py, j1 = (sy + 1) * ny / py;
      for (int j = j0; j < j1; ++j)
        for (int i = i0; i < i1; ++i) {
          const int nint = (i > 0) + (i < nx - 1) + (j > 0) + (j < ny - 1);
          ptr[g + 1] = ptr[g] + 16 * (1 + nint);
          ++g;
        }
    }
  const int64_t nnz = ptr[ne], ntiles = ne / 64;
  // own-data arrays of the same mesh (element g at square (i, j): vertex ids j (nx + 1) + i ..., neighbour ids)
  std::vector<int> evh(4 * ne), nbh(4 * ne);
  std::vector<unsigned> fih(ne, 0x2301u);
  std::vector<double> tenh(ne, 1.0), vxh(2 * int64_t(nx + 1) * (ny + 1), 0.5);
  {
    std::vector<int64_t> id(ne);
    int64_t q = 0;
    for (int sx = 0; sx < px; ++sx)
      for (int sy = 0; sy < py; ++sy)
        for (int j = sy * ny / py; j < (sy + 1) * ny / py; ++j)
          for (int i = sx * nx / px; i < (sx + 1) * nx / px; ++i) id[int64_t(j) * nx + i] = q++;
    for (int j = 0; j < ny; ++j)
      for (int i = 0; i < nx; ++i) {
        const int64_t e = id[int64_t(j) * nx + i];
        const int v00 = j * (nx + 1) + i;
        evh[0 * ne + e] = v00; evh[1 * ne + e] = v00 + 1; evh[2 * ne + e] = v00 + nx + 1; evh[3 * ne + e] = v00 + nx + 2;
        nbh[0 * ne + e] = i > 0 ? int(id[int64_t(j) * nx + i - 1]) : -1;
        nbh[1 * ne + e] = i < nx - 1 ? int(id[int64_t(j) * nx + i + 1]) : -1;
        nbh[2 * ne + e] = j > 0 ? int(id[int64_t(j - 1) * nx + i]) : -1;
        nbh[3 * ne + e] = j < ny - 1 ? int(id[int64_t(j + 1) * nx + i]) : -1;
      }
  }
  Mesh mesh;
  {
    int *a, *b;
    unsigned* c;
    double *d, *v;
    hipMalloc(&a, evh.size() * 4); hipMemcpy(a, evh.data(), evh.size() * 4, hipMemcpyHostToDevice);
    hipMalloc(&b, nbh.size() * 4); hipMemcpy(b, nbh.data(), nbh.size() * 4, hipMemcpyHostToDevice);
    hipMalloc(&c, fih.size() * 4); hipMemcpy(c, fih.data(), fih.size() * 4, hipMemcpyHostToDevice);
    hipMalloc(&d, tenh.size() * 8); hipMemcpy(d, tenh.data(), tenh.size() * 8, hipMemcpyHostToDevice);
    hipMalloc(&v, vxh.size() * 8); hipMemcpy(v, vxh.data(), vxh.size() * 8, hipMemcpyHostToDevice);
    mesh = Mesh{a, b, c, d, v, ne};
  }
  const double bytes = double(nnz) * 8;
  printf("C4 value array: %lld elements, %lld tiles, %lld values = %.4f GB\n", (long long)ne, (long long)ntiles,
         (long long)nnz, bytes * 1e-9);
  int64_t* dptr;
  double* out;
  hipMalloc(&dptr, (ne + 1) * 8);
  hipMemcpy(dptr, ptr.data(), (ne + 1) * 8, hipMemcpyHostToDevice);
  hipMalloc(&out, nnz * 8 + 4096);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipFuncSetAttribute((const void*)waveimg<64>, hipFuncAttributeMaxDynamicSharedMemorySize, 40960);
  hipFuncSetAttribute((const void*)coop<2, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 81920);
  hipFuncSetAttribute((const void*)coop<4, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 81920);
  hipFuncSetAttribute((const void*)coop<4, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  hipFuncSetAttribute((const void*)coop<8, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  hipFuncSetAttribute((const void*)waveimgL<64>, hipFuncAttributeMaxDynamicSharedMemorySize, 40960);
  hipFuncSetAttribute((const void*)coopL<8, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  hipFuncSetAttribute((const void*)coopL<4, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 81920);
  hipFuncSetAttribute((const void*)waveimgNP<64, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 40960);
  hipFuncSetAttribute((const void*)waveimgNP<64, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 40960);
#define ATTR(WW, NN) \
  hipFuncSetAttribute((const void*)coopC<WW, NN, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 20480 * WW); \
  hipFuncSetAttribute((const void*)coopC<WW, NN, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 20480 * WW);
  ATTR(1, 0) ATTR(1, 512) ATTR(1, 1024) ATTR(1, 1536) ATTR(2, 0) ATTR(2, 512) ATTR(2, 1024) ATTR(2, 1536)
  ATTR(4, 0) ATTR(4, 512) ATTR(4, 1024) ATTR(4, 1536) ATTR(8, 0) ATTR(8, 512) ATTR(8, 1024) ATTR(8, 1536)
#undef ATTR
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto time = [&](const char* name, auto launch) {
    launch();
    hipDeviceSynchronize();
    float ms[3];
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      for (int r = 0; r < 20; ++r) launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms[rep], e0, e1);
      ms[rep] /= 20;
    }
    std::sort(ms, ms + 3);
    printf("%-44s best %7.4f ms  median %7.4f ms  %5.2f TB/s\n", name, ms[0], ms[1], bytes / (ms[0] * 1e-3) / 1e12);
    fflush(stdout);
  };
  // (the half-image kernel: 8 workgroups per CU = 2 waves per SIMD at 20 KB; whole tiles 4 per CU at 40 KB)
  const bool skip_k = argc > 2 && atoi(argv[2]) == 1;   // argv[2] == 1: no XCD-interleaving (K) sweeps
  for (int pass = 0; pass < passes; ++pass) {
    printf("-- pass %d (%d CUs)\n", pass, cus);
    {
      const int gnp = int(8 * ((ntiles + 7) / 8));
      time("NP half20 eighths-remapped, stores only", [&] { waveimgNP<32, false><<<gnp, 64, 20480>>>(out, dptr, ntiles, mesh); });
      time("NP half20 eighths-remapped, + own loads", [&] { waveimgNP<32, true><<<gnp, 64, 20480>>>(out, dptr, ntiles, mesh); });
      time("NP whole40 eighths-remapped, stores only", [&] { waveimgNP<64, false><<<gnp, 64, 40960>>>(out, dptr, ntiles, mesh); });
      time("NP whole40 eighths-remapped, + own loads", [&] { waveimgNP<64, true><<<gnp, 64, 40960>>>(out, dptr, ntiles, mesh); });
      time("fill4kE  nt, chunks remapped to XCD eighths", [&] { fill4kE<<<int(8 * ((nnz / 512 + 7) / 8)), 256>>>(out, nnz); });
      time("fill4k   nt (same bytes)", [&] { fill4k<true><<<int((nnz + 511) / 512), 256>>>(out, nnz); });
      time("half20   1 wave/WG, 8 WG/CU (2 waves/SIMD)", [&] { waveimg<32><<<cus * 8, 64, 20480>>>(out, dptr, ntiles); });
      time("half20+own  8 WG/CU (own records + vertex rows)", [&] { waveimgL<32><<<cus * 8, 64, 20480>>>(out, dptr, ntiles, mesh); });
      if (argc > 3 && argv[3][0] == 'n') continue;
    }
    if (argc > 3) {   // the compute model: W x NC, with / without stores
      const int NCs[] = {0, 512, 1024, 1536};
      auto run = [&](int W, int nci, bool st) {
        char nm[96];
        snprintf(nm, sizeof nm, "model W=%d NC=%-4d %s", W, NCs[nci], st ? "stores  " : "no store");
        const int g = cus * (8 / W), sh = 20480 * W, nt = 64 * W;
#define MODEL(WW, II) if (W == WW && nci == II) time(nm, [&] { if (st) coopC<WW, NCs_##II, true><<<g, nt, sh>>>(out, dptr, ntiles, mesh); \
                                                           else coopC<WW, NCs_##II, false><<<g, nt, sh>>>(out, dptr, ntiles, mesh); });
        constexpr int NCs_0 = 0, NCs_1 = 512, NCs_2 = 1024, NCs_3 = 1536;
        MODEL(1, 0) MODEL(1, 1) MODEL(1, 2) MODEL(1, 3) MODEL(2, 0) MODEL(2, 1) MODEL(2, 2) MODEL(2, 3)
        MODEL(4, 0) MODEL(4, 1) MODEL(4, 2) MODEL(4, 3) MODEL(8, 0) MODEL(8, 1) MODEL(8, 2) MODEL(8, 3)
#undef MODEL
      };
      for (int nci = 0; nci < 4; ++nci)
        for (int W : {1, 2, 4, 8}) {
          run(W, nci, true);
          run(W, nci, false);
        }
      continue;
    }
    time("half20+own  8 WG/CU (own records + vertex rows)", [&] { waveimgL<32><<<cus * 8, 64, 20480>>>(out, dptr, ntiles, mesh); });
    time("whole40+own 4 WG/CU", [&] { waveimgL<64><<<cus * 4, 64, 40960>>>(out, dptr, ntiles, mesh); });
    time("coop8_4+own 1 WG/CU", [&] { coopL<8, 4><<<cus, 512, 163840>>>(out, dptr, ntiles, mesh); });
    time("coop4_2+own 2 WG/CU", [&] { coopL<4, 2><<<cus * 2, 256, 81920>>>(out, dptr, ntiles, mesh); });
    for (int64_t K : {1, 2, 4, 8, 16, 64, 256}) {
      if (skip_k) break;
      char nm[96];
      snprintf(nm, sizeof nm, "half20 K=%-4lld XCD-interleaved, 8 WG/CU", (long long)K);
      time(nm, [&] { waveimgK<32><<<cus * 8, 64, 20480>>>(out, dptr, ntiles, K); });
    }
    for (int64_t K : {1, 8, 16}) {
      if (skip_k) break;
      char nm[96];
      snprintf(nm, sizeof nm, "whole40 K=%-4lld XCD-interleaved, 4 WG/CU", (long long)K);
      time(nm, [&] { waveimgK<64><<<cus * 4, 64, 40960>>>(out, dptr, ntiles, K); });
    }
    if (!skip_k) time("half20   one tile per workgroup (grid = tiles)", [&] { waveimgK<32><<<int(ntiles), 64, 20480>>>(out, dptr, ntiles, 0); });
    if (!skip_k) time("whole40  one tile per workgroup (grid = tiles)", [&] { waveimgK<64><<<int(ntiles), 64, 40960>>>(out, dptr, ntiles, 0); });
    for (int64_t K : {1, 16, 640}) {
      if (skip_k) break;
      char nm[96];
      snprintf(nm, sizeof nm, "fillK1k K=%-4lld KB XCD-interleaved, 8 WG/CU", (long long)K);
      time(nm, [&] { fillK1k<<<cus * 8, 64>>>(out, nnz, K); });
    }
    time("half20   1 wave/WG, 8 WG/CU (2 waves/SIMD)", [&] { waveimg<32><<<cus * 8, 64, 20480>>>(out, dptr, ntiles); });
    time("half20   1 wave/WG, 5 WG/CU", [&] { waveimg<32><<<cus * 5, 64, 20480>>>(out, dptr, ntiles); });
    time("half20   1 wave/WG, 4 WG/CU (1 wave/SIMD)", [&] { waveimg<32><<<cus * 4, 64, 20480>>>(out, dptr, ntiles); });
    time("whole40  1 wave/WG, 4 WG/CU (1 wave/SIMD)", [&] { waveimg<64><<<cus * 4, 64, 40960>>>(out, dptr, ntiles); });
    time("coop2_1  2 waves, 1 tile, 4 WG/CU", [&] { coop<2, 1><<<cus * 4, 128, 40960>>>(out, dptr, ntiles); });
    time("coop2_2  2 waves, 2 tiles, 2 WG/CU", [&] { coop<2, 2><<<cus * 2, 128, 81920>>>(out, dptr, ntiles); });
    time("coop4_2  4 waves, 2 tiles, 2 WG/CU", [&] { coop<4, 2><<<cus * 2, 256, 81920>>>(out, dptr, ntiles); });
    time("coop4_4  4 waves, 4 tiles, 1 WG/CU", [&] { coop<4, 4><<<cus * 1, 256, 163840>>>(out, dptr, ntiles); });
    time("coop8_4  8 waves, 4 tiles, 1 WG/CU", [&] { coop<8, 4><<<cus * 1, 512, 163840>>>(out, dptr, ntiles); });
    time("fill4k   nt (same bytes)", [&] { fill4k<true><<<int((nnz + 511) / 512), 256>>>(out, nnz); });
    time("fill4k   plain (same bytes)", [&] { fill4k<false><<<int((nnz + 511) / 512), 256>>>(out, nnz); });
    time("fillE1k  persistent XCD eighths, 8 WG/CU", [&] { fillE1k<<<cus * 8, 64>>>(out, nnz); });
  }
  hipFree(out);
  hipFree(dptr);
  return 0;
}
