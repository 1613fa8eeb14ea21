// Write-stream microbenchmark, part 7: the C4 (Q1) store phase -- every wave streams its own 40 KB tile
// image, XCD eighths, 4 waves per CU (wstream6 "E") -- with the tile's own-data reads laid out as the
// production kernel reads them, against packed alternatives:
//   SOA14  14 SoA segments per tile, as Q1PwcPolicy::load_own: 8 coordinate rows (f64), 4 neighbour rows
//          (i32), face info (u32), the per-element tensor (f64) = 92 B per element
//   SOA23  23 dword rows (wstream6's reads-before-stores)
//   AOS96  one element-major record of 96 B per element (geometry + topology + tensor), 6 x 16 B per lane
//   AOS2   an 80 B geometry/topology record (5 x 16 B per lane) + the tensor row (f64 SoA)
//   AOS96L like AOS96 but the tile's 6 KB read wave-coalesced (instruction k = bytes [1 KB k, 1 KB (k+1)))
//          and handed to the lanes through LDS
// each with the next tile's reads issued before this tile's stores (production order), plus stores only.
// Build: hipcc -O3 --offload-arch=gfx950 -Wno-unused-result wstream7.hip -o wstream7
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dvec2 __attribute__((ext_vector_type(2)));
typedef int ivec4 __attribute__((ext_vector_type(4)));

constexpr int RB = 80, IMG = 64 * RB, ST = IMG / 128;
enum { NONE = 0, SOA14 = 1, SOA23 = 2, AOS96 = 3, AOS2 = 4, AOS96L = 5 };

struct Rd {
  double d[10];
  int i[12];
};

template <int MODE>
__device__ __forceinline__ void load(const char* in, long n, long tile, int lane, double* lrd, Rd& r)
{
  const long e = tile * 64 + lane;
  if constexpr (MODE == SOA14) {
    const double* c = reinterpret_cast<const double*>(in);
#pragma unroll
    for (int k = 0; k < 8; ++k) r.d[k] = c[k * n + e];
    const int* nb = reinterpret_cast<const int*>(c + 8 * n);
#pragma unroll
    for (int k = 0; k < 5; ++k) r.i[k] = nb[k * n + e];
    r.d[8] = reinterpret_cast<const double*>(nb + 5 * n)[e];
  } else if constexpr (MODE == SOA23) {
    const int* c = reinterpret_cast<const int*>(in);
#pragma unroll
    for (int k = 0; k < 23; ++k) (k < 12 ? r.i[k] : reinterpret_cast<int*>(r.d)[k - 12]) = c[k * n + e];
  } else if constexpr (MODE == AOS96 || MODE == AOS2) {
    constexpr int NV = MODE == AOS96 ? 6 : 5;
    const ivec4* p = reinterpret_cast<const ivec4*>(in + e * (16 * NV));
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const ivec4 v = p[k];
      r.i[2 * k] = v.x ^ v.y;
      r.i[2 * k + 1] = v.z ^ v.w;
    }
    if constexpr (MODE == AOS2) r.d[8] = reinterpret_cast<const double*>(in + n * 80)[e];
  } else if constexpr (MODE == AOS96L) {   // wave-coalesced 6 KB, then each lane reads its record from LDS
    const ivec4* p = reinterpret_cast<const ivec4*>(in + tile * 64 * 96);
    ivec4* l = reinterpret_cast<ivec4*>(lrd);
#pragma unroll
    for (int k = 0; k < 6; ++k) l[k * 64 + lane] = p[k * 64 + lane];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const ivec4 v = l[lane * 6 + k];
      r.i[2 * k] = v.x ^ v.y;
      r.i[2 * k + 1] = v.z ^ v.w;
    }
  }
}

template <int MODE>
__device__ __forceinline__ int fold(const Rd& r)
{
  int acc = 0;
#pragma unroll
  for (int k = 0; k < 12; ++k) acc += r.i[k];
#pragma unroll
  for (int k = 0; k < 10; ++k) acc += int(r.d[k]);
  return acc;
}

template <int MODE>
__global__ void __launch_bounds__(64, 1) own(double* out, const char* in, long ntiles, long n)
{
  __shared__ __attribute__((aligned(16))) double lds[MODE == AOS96L ? IMG + 6 * 64 * 2 : IMG];   // 40 KB: 4 waves per CU
  double* lrd = lds + IMG;
  const int lane = threadIdx.x;
  for (int j = 0; j < RB; ++j) lds[lane * RB + j] = j;
  __builtin_amdgcn_wave_barrier();
  const long G = gridDim.x, b = blockIdx.x, x = b & 7, w = b >> 3, gx = G >> 3;
  const long s0 = (ntiles * x) / 8, s1 = (ntiles * (x + 1)) / 8;
  long t = s0 + w;
  if (t >= s1) return;
  Rd cur{};
  int acc = 0;
  if (MODE) load<MODE>(in, n, t, lane, lrd, cur);
  for (; t < s1; t += gx) {
    Rd nx{};
    const long tn = t + gx < s1 ? t + gx : t;
    if (MODE) load<MODE>(in, n, tn, lane, lrd, nx);
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + t * IMG, (short)0, IMG * 8, 0x00020000);
#pragma unroll
    for (int k = 0; k < ST; ++k) {
      const int idx = 2 * (lane + 64 * k);
      const dvec2 v = *reinterpret_cast<const dvec2*>(lds + idx);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), rs, idx * 8, 0, 2);
    }
    if (MODE) {
      acc += fold<MODE>(cur);
      cur = nx;
    }
  }
  if (MODE && acc == 123456789) out[0] = acc;
}

int main()
{
  const long ntiles = 66000, n = ntiles * 64, nv = ntiles * IMG;
  double* out;
  char* in;
  (void)hipMalloc(&out, (nv + 64) * 8);
  (void)hipMalloc(&in, n * 128);
  (void)hipMemset(in, 0, n * 128);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  auto time = [&](const char* name, double rbytes, auto launch) {
    launch(); (void)hipDeviceSynchronize();
    float best = 1e9, sum = 0;
    for (int rep = 0; rep < 5; ++rep) {
      (void)hipEventRecord(e0);
      for (int r = 0; r < 20; ++r) launch();
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1); ms /= 20;
      best = ms < best ? ms : best; sum += ms;
    }
    const double wb = double(nv) * 8;
    printf("%-30s best %8.4f ms  mean %8.4f ms  %6.2f TB/s (read %5.3f GB)\n", name, best, sum / 5,
           (wb + rbytes) / (best * 1e-3) / 1e12, rbytes / 1e9);
    fflush(stdout);
  };
  for (int pass = 0; pass < 2; ++pass) {
    printf("-- pass %d (%d CUs, %ld tiles of %d KB)\n", pass, cus, ntiles, IMG * 8 / 1024);
#define RUN(M, RBY, NAME) time(NAME, double(RBY) * n, [&] { hipLaunchKernelGGL((own<M>), dim3(cus * 4), dim3(64), 0, 0, out, in, ntiles, n); })
    RUN(NONE, 0, "stores only");
    RUN(SOA14, 92, "SOA14 (production layout)");
    RUN(SOA23, 92, "SOA23 (wstream6)");
    RUN(AOS96, 96, "AOS96 lane records");
    RUN(AOS2, 88, "AOS2 80 B record + tensor row");
    RUN(AOS96L, 96, "AOS96L via LDS (46 KB: 3/CU)");
  }
  return 0;
}
