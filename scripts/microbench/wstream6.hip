// Write-stream microbenchmark, part 6: the C4 (Q1) store phase -- every wave streams its own 40 KB tile image
// (64 elements x 80 doubles) -- under different tile -> wave assignments, and with the per-tile own-data
// reads of the Q1 kernel (23 dwords per element from SoA arrays, the next tile's, issued before the stores).
//   E  XCD eighths, concurrent waves on consecutive tiles (production schedule)
//   B  XCD eighths, each wave a contiguous block of tiles (concurrent waves ~ eighth / 128 tiles apart)
//   R  global round robin (tile = b + k G)
//   S  E with each wave starting its 40 stores at chunk (w mod 40) and wrapping (staggered offsets)
//   F1 reference fill: XCD eighths, 1 KB per wave per round
// SKEW = 0: 128-B aligned tile bases (C4: every Q1 row block is a multiple of 16 doubles); SKEW = 10: the 80 B
// offset of the earlier C2 studies.  RD = 2: the next tile's reads issued after this tile's stores.
// Build: hipcc -O3 --offload-arch=gfx950 -Wno-unused-result wstream6.hip -o wstream6
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dvec2 __attribute__((ext_vector_type(2)));
typedef int ivec4 __attribute__((ext_vector_type(4)));

constexpr int RB = 80, IMG = 64 * RB, ST = IMG / 128, NRD = 23;

__device__ __forceinline__ void sched(int mode, long ntiles, long& t, long& te, long& ts)
{
  const long G = gridDim.x, b = blockIdx.x, x = b & 7, w = b >> 3, gx = G >> 3;
  const long s0 = (ntiles * x) / 8, s1 = (ntiles * (x + 1)) / 8;
  if (mode == 1) {        // B
    t = s0 + ((s1 - s0) * w) / gx; te = s0 + ((s1 - s0) * (w + 1)) / gx; ts = 1;
  } else if (mode == 2) { // R
    t = b; te = ntiles; ts = G;
  } else {                // E, S
    t = s0 + w; te = s1; ts = gx;
  }
}

template <int MODE, int RD, int SKEW>
__global__ void __launch_bounds__(64, 1) own(double* out, const int* in, long ntiles, long n)
{
  __shared__ __attribute__((aligned(16))) double lds[IMG];
  const int lane = threadIdx.x;
  for (int j = 0; j < RB; ++j) lds[lane * RB + j] = j;
  __builtin_amdgcn_wave_barrier();
  long t, te, ts;
  sched(MODE == 3 ? 0 : MODE, ntiles, t, te, ts);
  const int rot = MODE == 3 ? int((blockIdx.x >> 3) % ST) : 0;
  int acc = 0, cur[NRD];
  if (RD) {
#pragma unroll
    for (int r = 0; r < NRD; ++r) cur[r] = in[long(r) * n + t * 64 + lane];
  }
  for (; t < te; t += ts) {
    int nx[NRD];
    const long tn = t + ts < te ? t + ts : t;
    if (RD == 1) {   // the next tile's own data, issued before this tile's stores (production order)
#pragma unroll
      for (int r = 0; r < NRD; ++r) nx[r] = in[long(r) * n + tn * 64 + lane];
    }
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + SKEW + t * IMG, (short)0, IMG * 8, 0x00020000);
#pragma unroll
    for (int k = 0; k < ST; ++k) {
      int kk = k + rot;
      kk = kk < ST ? kk : kk - ST;
      const int idx = 2 * (lane + 64 * kk);
      const dvec2 v = *reinterpret_cast<const dvec2*>(lds + idx);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), rs, idx * 8, 0, 2);
    }
    if (RD == 2) {
#pragma unroll
      for (int r = 0; r < NRD; ++r) nx[r] = in[long(r) * n + tn * 64 + lane];
    }
    if (RD) {
#pragma unroll
      for (int r = 0; r < NRD; ++r) { acc += cur[r]; cur[r] = nx[r]; }
    }
  }
  if (RD && acc == 123456789) out[0] = acc;
}

template <int SKEW>
__global__ void __launch_bounds__(64, 1) fill1(double* out, long nch)
{
  const long G = gridDim.x, b = blockIdx.x, x = b & 7, w = b >> 3, gx = G >> 3;
  const dvec2 v = {1.0, 2.0};
  for (long c = (nch * x) / 8 + w; c < (nch * (x + 1)) / 8; c += gx) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + SKEW + c * 128, (short)0, 1024, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), rs, threadIdx.x * 16, 0, 2);
  }
}

int main()
{
  const long ntiles = 66000, n = ntiles * 64, nv = ntiles * IMG;
  double* out;
  int* in;
  (void)hipMalloc(&out, (nv + 64) * 8);
  (void)hipMalloc(&in, long(NRD) * n * 4);
  (void)hipMemset(in, 0, long(NRD) * n * 4);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  auto time = [&](const char* name, double bytes, auto launch) {
    launch(); (void)hipDeviceSynchronize();
    float best = 1e9, sum = 0;
    for (int rep = 0; rep < 5; ++rep) {
      (void)hipEventRecord(e0);
      for (int r = 0; r < 20; ++r) launch();
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1); ms /= 20;
      best = ms < best ? ms : best; sum += ms;
    }
    printf("%-34s best %8.4f ms  mean %8.4f ms  %6.2f TB/s\n", name, best, sum / 5, bytes / (best * 1e-3) / 1e12);
    fflush(stdout);
  };
  const double wb = double(nv) * 8, rb = double(NRD) * n * 4;
  for (int pass = 0; pass < 2; ++pass) {
    printf("-- pass %d (%d CUs, %ld tiles of %d KB)\n", pass, cus, ntiles, IMG * 8 / 1024);
#define FILL(SK, NAME) time(NAME, wb, [&] { hipLaunchKernelGGL((fill1<SK>), dim3(cus * 4), dim3(64), 0, 0, out, nv / 128); })
#define OWN(M, RD, SK, WG, NAME) time(NAME, wb + (RD ? rb : 0.0), [&] { \
    hipLaunchKernelGGL((own<M, RD, SK>), dim3(cus * WG), dim3(64), 0, 0, out, in, ntiles, n); })
    FILL(0, "F1 fill 1 KB/wave-round x4 aligned");
    FILL(10, "F1 fill 1 KB/wave-round x4 skew80");
    OWN(0, 0, 0, 4, "E  stores only x4");
    OWN(1, 0, 0, 4, "B  stores only x4");
    OWN(2, 0, 0, 4, "R  stores only x4");
    OWN(3, 0, 0, 4, "S  stores only x4");
    OWN(0, 0, 0, 3, "E  stores only x3");
    OWN(0, 0, 0, 2, "E  stores only x2");
    OWN(0, 1, 0, 4, "E  reads-before-stores x4");
    OWN(0, 2, 0, 4, "E  reads-after-stores x4");
    OWN(2, 1, 0, 4, "R  reads-before-stores x4");
    OWN(3, 1, 0, 4, "S  reads-before-stores x4");
    OWN(3, 2, 0, 4, "S  reads-after-stores x4");
    OWN(0, 0, 10, 4, "E  stores only x4 skew80");
  }
  return 0;
}
