// dune-hdd_amd/csrc/kernels/shard.hip
//
// Sharded BlockSWIPDG behind the C ABI (SURVEY.md 8(b) hdd_block_assemble_sharded, 8(e)).
//
// The reference assembles BlockSWIPDG sequentially over subdomains (block-swipdg.hh:271, 334): the local
// operator of ss, the boundary terms of a domain-boundary subdomain (assemble_boundary_contributions,
// 1136-1179) and, for each neighbour nn > ss, the SWIPDG::Inner coupling into A_ss, A_ss,nn, A_nn,ss, A_nn
// (assemble_coupling_contributions, 1270-1326).  Here one rank (process or thread, one GPU each) owns a
// contiguous subdomain range and writes exactly the rows of its elements -- the rows of A_ss and A_ss,nn
// (block-swipdg.hh:355-382) -- computing both sides of every face it touches (owner-computes), so no
// matrix entry is ever summed across ranks.  The only exchange is the face halo: the per-element records
// (diffusion tensor, per-element diffusion factors [, vertex coordinates]) of the ghost elements.
//
// One step: pack (one kernel, every peer) -> post the exchange (RCCL group send/recv on the
// communicator's transfer stream, or a host transport) -> interior 64-element tiles on the caller's
// stream while the halo is in flight -> stream waits for the receives -> unpack into the ghost columns
// -> the tiles that touch a ghost.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "hdd.h"
#include "../host/hdd_internal.hh"

using hdd::set_error;

namespace {

int hip_fail(hipError_t e, const char* where)
{
  return set_error(HDD_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

// Events that only order two streams of ONE device (the step's side stream against `stream`, RCCL's transfer
// stream back into `stream`): the data both sides touch stays on that device, so a device-scope release /
// acquire is enough.  A default event's record is a system-scope release -- an L2 write-back of everything the
// previous tile launch left dirty -- which sits between two launches of back-to-back steps (C4 N = 8 one-card
// trace, profiles/r04/q_btb/: 12.5 us of 93 us per step with nothing running).  Events another device waits on
// (the device transport's "packed" = comm->ready, read by peer copies; RCCL may read send buffers from a peer)
// keep the system fence.  HDD_EVENT_SYSTEM_FENCE=1 restores it everywhere (A/B).
unsigned local_event_flags()
{
  static const bool sys = getenv("HDD_EVENT_SYSTEM_FENCE") != nullptr;
  return sys ? hipEventDisableTiming : hipEventDisableTiming | hipEventDisableSystemFence;
}

// ------------------------------------------------------------------------------------------------
// RCCL, resolved at run time: in a PyTorch process this is torch's own librccl (already loaded, found
// through the library's rpath), so the process holds one RCCL and one HIP runtime.
// ------------------------------------------------------------------------------------------------
struct RcclApi {
  bool ok = false;
  std::string err;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

RcclApi load_rccl()
{
  RcclApi r;
  void* h = nullptr;
  for (const char* name : {"librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so.1"}) {
    h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
    if (h) break;
  }
  if (!h)
    for (const char* name : {"librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so.1"}) {
      h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
      if (h) break;
    }
  if (!h) {
    const char* e = dlerror();
    r.err = std::string("librccl not found: ") + (e ? e : "");
    return r;
  }
  bool all = true;
  auto sym = [&](auto& fp, const char* name) {
    fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
    if (!fp) {
      all = false;
      r.err += std::string(" missing ") + name;
    }
  };
  sym(r.GetUniqueId, "ncclGetUniqueId");
  sym(r.CommInitRank, "ncclCommInitRank");
  sym(r.CommDestroy, "ncclCommDestroy");
  sym(r.GroupStart, "ncclGroupStart");
  sym(r.GroupEnd, "ncclGroupEnd");
  sym(r.Send, "ncclSend");
  sym(r.Recv, "ncclRecv");
  sym(r.GetErrorString, "ncclGetErrorString");
  r.ok = all;
  return r;
}

const RcclApi& rccl()
{
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] { api = load_rccl(); });
  return api;
}

int nccl_fail(ncclResult_t r, const char* where)
{
  const char* s = rccl().GetErrorString ? rccl().GetErrorString(r) : "?";
  return set_error(HDD_ERR_HIP, std::string(where) + ": RCCL error " + std::to_string(int(r)) + " (" + s + ")");
}

// ------------------------------------------------------------------------------------------------
// halo pack / unpack: message of peer p = [rows][count_p] doubles at buf + R * prefix[p]
// ------------------------------------------------------------------------------------------------
constexpr int SH_MAX_ARR = 16;
constexpr int SH_MAX_PEERS = 64;

struct HaloArgs {
  double* arr[SH_MAX_ARR];             // element-column arrays [rows][ld]
  int32_t row_first[SH_MAX_ARR + 1];   // first halo row of each array
  int32_t n_arrays, n_peers;
  int64_t ld;
  int64_t prefix[SH_MAX_PEERS + 1];    // element prefix over the peers' messages
  int64_t col0[SH_MAX_PEERS];          // unpack: first ghost column of peer p
  const int32_t* idx;                  // pack: concatenated send lists (local element ids)
  double* buf;
};

__device__ __forceinline__ void halo_slot(const HaloArgs& a, int64_t t, int& p, int& arr, int64_t& rr, int64_t& i)
{
  const int R = a.row_first[a.n_arrays];
  p = 0;
  while (p + 1 < a.n_peers && int64_t(R) * a.prefix[p + 1] <= t) ++p;
  const int64_t cnt = a.prefix[p + 1] - a.prefix[p];
  const int64_t loc = t - int64_t(R) * a.prefix[p];
  const int64_t r = loc / cnt;
  i = loc - r * cnt;
  arr = 0;
  while (arr + 1 < a.n_arrays && a.row_first[arr + 1] <= r) ++arr;
  rr = r - a.row_first[arr];
}

__global__ void __launch_bounds__(256) halo_pack_kernel(const HaloArgs a)
{
  const int64_t total = int64_t(a.row_first[a.n_arrays]) * a.prefix[a.n_peers];
  for (int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; t < total; t += int64_t(gridDim.x) * blockDim.x) {
    int p, arr;
    int64_t rr, i;
    halo_slot(a, t, p, arr, rr, i);
    a.buf[t] = a.arr[arr][rr * a.ld + a.idx[a.prefix[p] + i]];
  }
}

__global__ void __launch_bounds__(256) halo_unpack_kernel(const HaloArgs a)
{
  const int64_t total = int64_t(a.row_first[a.n_arrays]) * a.prefix[a.n_peers];
  for (int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; t < total; t += int64_t(gridDim.x) * blockDim.x) {
    int p, arr;
    int64_t rr, i;
    halo_slot(a, t, p, arr, rr, i);
    a.arr[arr][rr * a.ld + a.col0[p] + i] = a.buf[t];
  }
}

template <class T>
hipError_t upload(T** d, const std::vector<T>& h)
{
  *d = nullptr;
  if (h.empty()) return hipSuccess;
  hipError_t e = hipMalloc(d, h.size() * sizeof(T));
  if (e != hipSuccess) return e;
  return hipMemcpy(*d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice);
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// in-process device transport (hdd_device_hub): several ranks of one process (one thread each, any devices)
// exchanging device buffers with the stream / event schedule of an RCCL group send/recv.  Per directed pair
// (src, dst) a channel holds the sender's latest publication -- its message list and its "packed" event (the
// send buffers are complete) -- and the receiver's "consumed" event (its copies out of them are complete).
// ------------------------------------------------------------------------------------------------
struct hdd_device_hub {
  struct Channel {
    uint64_t sent = 0, consumed = 0;     // publications by src / publications dst has copied out of
    std::vector<std::pair<const double*, int64_t>> msgs;
    hipEvent_t packed = nullptr;         // src's event after its packs
    hipEvent_t copied = nullptr;         // dst's event after its copies out of publication `consumed`
  };
  int32_t nranks = 0;
  std::mutex m;
  std::condition_variable cv;
  std::vector<Channel> ch;               // [src * nranks + dst]
  std::string failed;                    // first protocol error (every waiting rank returns it)
  int refs = 1;
  double timeout_s = 120.0;
  // error injection (hdd_device_hub_stall): the next post of rank `stall_rank` gates its sends behind a device-side
  // wait for a host word (a peer whose sends never complete, bounded by stall_s), released by hdd_device_hub_release
  int32_t stall_rank = -1;
  double stall_s = 0.0;
  uint32_t* gate = nullptr;              // pinned host word (device-visible): 0 = closed
};

// The injected stall: one wave spins (s_sleep between polls) until the host opens the gate or max_ticks of the
// 100 MHz real-time counter have passed -- every launch ends by itself.
__global__ void __launch_bounds__(64) hub_gate_kernel(const uint32_t* gate, uint64_t max_ticks)
{
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u &&
         __builtin_amdgcn_s_memrealtime() - t0 < max_ticks)
    __builtin_amdgcn_s_sleep(100);
}

static void hub_release(hdd_device_hub* h)
{
  if (!h) return;
  bool last;
  {
    std::lock_guard<std::mutex> lk(h->m);
    last = --h->refs == 0;
  }
  if (last) {
    if (h->gate) (void)hipHostFree(h->gate);
    delete h;
  }
}

extern "C" int hdd_device_hub_create(int32_t nranks, hdd_device_hub** out)
{
  if (!out || nranks < 1) return set_error(HDD_ERR_INVALID, "hdd_device_hub_create: invalid argument");
  auto* h = new hdd_device_hub;
  h->nranks = nranks;
  h->ch.resize(size_t(nranks) * size_t(nranks));
  *out = h;
  return HDD_OK;
}

extern "C" void hdd_device_hub_destroy(hdd_device_hub* hub) { hub_release(hub); }

extern "C" int hdd_device_hub_stall(hdd_device_hub* hub, int32_t rank, double max_seconds)
{
  if (!hub || rank < 0 || rank >= hub->nranks || !(max_seconds > 0.0) || max_seconds > 600.0)
    return set_error(HDD_ERR_INVALID, "hdd_device_hub_stall: invalid argument");
  std::lock_guard<std::mutex> lk(hub->m);
  if (!hub->gate) {
    const hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&hub->gate), 64, hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) {
      hub->gate = nullptr;
      return hip_fail(e, "hdd_device_hub_stall: gate word");
    }
  }
  __atomic_store_n(hub->gate, 0u, __ATOMIC_SEQ_CST);
  hub->stall_rank = rank;
  hub->stall_s = max_seconds;
  return HDD_OK;
}

extern "C" int hdd_device_hub_release(hdd_device_hub* hub)
{
  if (!hub) return set_error(HDD_ERR_INVALID, "hdd_device_hub_release: null hub");
  std::lock_guard<std::mutex> lk(hub->m);
  if (hub->gate) __atomic_store_n(hub->gate, 1u, __ATOMIC_SEQ_CST);
  hub->stall_rank = -1;
  return HDD_OK;
}

// ------------------------------------------------------------------------------------------------
// communicators
// ------------------------------------------------------------------------------------------------
struct hdd_comm {
  enum Kind { RCCL_OWNED, RCCL_WRAPPED, HOST, DEVICE } kind = HOST;
  int device = 0;
  ncclComm_t nccl = nullptr;
  hipStream_t xfer = nullptr;          // transfer stream (RCCL, DEVICE)
  hipEvent_t ready = nullptr, done = nullptr;
  bool posted = false;
  hdd_host_exchange_fn fn = nullptr;
  void* user = nullptr;
  double* pinned = nullptr;            // host staging (HOST)
  size_t pinned_doubles = 0;
  hdd_device_hub* hub = nullptr;       // DEVICE: the hub, this rank, one "copied" event per source rank
  int32_t rank = 0;
  std::vector<hipEvent_t> copied;
  hipEvent_t gated = nullptr;          // DEVICE, injected stall: the sends' event behind the gate
  std::vector<int32_t> last_peers;     // the peers of the last post (watchdog messages)
  hipStream_t direct = nullptr;        // RCCL: the caller's stream the last post ran on directly (serial step)
};

static int comm_rccl_streams(hdd_comm* c)
{
  hipError_t e = hipSetDevice(c->device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->xfer, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ready, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->done, local_event_flags());
  return e == hipSuccess ? HDD_OK : hip_fail(e, "hdd_comm: transfer stream / events");
}

extern "C" int hdd_rccl_get_unique_id(void* id)
{
  if (!id) return set_error(HDD_ERR_INVALID, "hdd_rccl_get_unique_id: null id");
  static_assert(sizeof(ncclUniqueId) == HDD_RCCL_ID_BYTES, "ncclUniqueId size");
  const RcclApi& R = rccl();
  if (!R.ok) return set_error(HDD_ERR_UNSUPPORTED, "hdd_rccl_get_unique_id: " + R.err);
  ncclUniqueId u;
  const ncclResult_t r = R.GetUniqueId(&u);
  if (r != ncclSuccess) return nccl_fail(r, "ncclGetUniqueId");
  std::memcpy(id, &u, sizeof(u));
  return HDD_OK;
}

extern "C" int hdd_comm_create_rccl(const void* id, int32_t nranks, int32_t rank, int32_t hip_device, hdd_comm** out)
{
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks)
    return set_error(HDD_ERR_INVALID, "hdd_comm_create_rccl: invalid argument");
  const RcclApi& R = rccl();
  if (!R.ok) return set_error(HDD_ERR_UNSUPPORTED, "hdd_comm_create_rccl: " + R.err);
  auto* c = new hdd_comm;
  c->kind = hdd_comm::RCCL_OWNED;
  c->device = hip_device;
  int rc = comm_rccl_streams(c);
  if (rc) {
    hdd_comm_destroy(c);
    return rc;
  }
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  const ncclResult_t r = R.CommInitRank(&c->nccl, nranks, u, rank);
  if (r != ncclSuccess) {
    c->nccl = nullptr;
    hdd_comm_destroy(c);
    return nccl_fail(r, "ncclCommInitRank");
  }
  *out = c;
  return HDD_OK;
}

extern "C" int hdd_comm_wrap_rccl(void* nccl_comm, int32_t hip_device, hdd_comm** out)
{
  if (!nccl_comm || !out) return set_error(HDD_ERR_INVALID, "hdd_comm_wrap_rccl: invalid argument");
  const RcclApi& R = rccl();
  if (!R.ok) return set_error(HDD_ERR_UNSUPPORTED, "hdd_comm_wrap_rccl: " + R.err);
  auto* c = new hdd_comm;
  c->kind = hdd_comm::RCCL_WRAPPED;
  c->device = hip_device;
  c->nccl = static_cast<ncclComm_t>(nccl_comm);
  int rc = comm_rccl_streams(c);
  if (rc) {
    hdd_comm_destroy(c);
    return rc;
  }
  *out = c;
  return HDD_OK;
}

extern "C" int hdd_comm_create_host(hdd_host_exchange_fn fn, void* user, int32_t hip_device, hdd_comm** out)
{
  if (!fn || !out) return set_error(HDD_ERR_INVALID, "hdd_comm_create_host: invalid argument");
  auto* c = new hdd_comm;
  c->kind = hdd_comm::HOST;
  c->device = hip_device;
  c->fn = fn;
  c->user = user;
  *out = c;
  return HDD_OK;
}

extern "C" int hdd_comm_create_device(hdd_device_hub* hub, int32_t rank, int32_t hip_device, hdd_comm** out)
{
  if (!hub || !out || rank < 0 || rank >= hub->nranks)
    return set_error(HDD_ERR_INVALID, "hdd_comm_create_device: invalid argument");
  auto* c = new hdd_comm;
  c->kind = hdd_comm::DEVICE;
  c->device = hip_device;
  c->rank = rank;
  int rc = comm_rccl_streams(c);
  hipError_t e = hipSuccess;
  c->copied.assign(size_t(hub->nranks), nullptr);
  for (auto& ev : c->copied)
    if (rc == HDD_OK && e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (rc == HDD_OK && e != hipSuccess) rc = hip_fail(e, "hdd_comm_create_device: events");
  if (rc) {
    hdd_comm_destroy(c);
    return rc;
  }
  {
    std::lock_guard<std::mutex> lk(hub->m);
    ++hub->refs;
  }
  c->hub = hub;
  *out = c;
  return HDD_OK;
}

extern "C" void hdd_comm_destroy(hdd_comm* c)
{
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->xfer) (void)hipStreamSynchronize(c->xfer);
  if (c->kind == hdd_comm::RCCL_OWNED && c->nccl && rccl().ok) (void)rccl().CommDestroy(c->nccl);
  if (c->ready) (void)hipEventDestroy(c->ready);
  if (c->done) (void)hipEventDestroy(c->done);
  for (hipEvent_t ev : c->copied)
    if (ev) (void)hipEventDestroy(ev);
  if (c->gated) (void)hipEventDestroy(c->gated);
  if (c->xfer) (void)hipStreamDestroy(c->xfer);
  if (c->pinned) (void)hipHostFree(c->pinned);
  hub_release(c->hub);
  delete c;
}

// DEVICE transport: the group send/recv of one rank.  On the transfer stream (which already waits for the packs
// on `stream`): for every source rank, wait for its packed event, copy its messages into the receive buffers,
// record "copied"; then wait for every destination's "copied" event, so that -- as after ncclGroupEnd -- the
// completion event covers the sends too and the next pack cannot overwrite a send buffer that is still read.
// Host side: publish this rank's sends, then block until each source has published (RCCL blocks on the device
// instead; a thread per rank makes the host rendezvous harmless).  Messages of one directed pair match in order,
// zero-count messages are skipped on both sides (as RCCL does).
static int device_post(hdd_comm* c, int32_t n_peers, const int32_t* peers, const double* const* d_send,
                       const int64_t* send_count, double* const* d_recv, const int64_t* recv_count)
{
  hdd_device_hub& H = *c->hub;
  const int32_t me = c->rank, n = H.nranks;
  std::map<int32_t, std::vector<std::pair<const double*, int64_t>>> out;
  std::map<int32_t, std::vector<std::pair<double*, int64_t>>> in;
  for (int32_t k = 0; k < n_peers; ++k) {
    if (peers[k] < 0 || peers[k] >= n || send_count[k] < 0 || recv_count[k] < 0)
      return set_error(HDD_ERR_INVALID, "hdd_comm_post: peer or count out of range (device transport)");
    if (send_count[k] > 0) out[peers[k]].emplace_back(d_send[k], send_count[k]);
    if (recv_count[k] > 0) in[peers[k]].emplace_back(d_recv[k], recv_count[k]);
  }
  const auto limit = std::chrono::duration<double>(H.timeout_s);
  auto fail = [&](std::unique_lock<std::mutex>& lk, const std::string& msg) {
    if (H.failed.empty()) H.failed = msg;
    lk.unlock();
    H.cv.notify_all();
    return set_error(HDD_ERR_INVALID, "hdd_comm_post (device transport): " + msg);
  };
  hipEvent_t packed_ev = c->ready;   // recorded on the pack stream by the caller; the transfer stream waits for it
  {
    std::lock_guard<std::mutex> lk(H.m);
    if (H.stall_rank == me && H.gate) {   // injected stall: the sends complete only once the gate opens
      if (!c->gated && hipEventCreateWithFlags(&c->gated, hipEventDisableTiming) != hipSuccess) c->gated = nullptr;
      uint32_t* dgate = nullptr;
      hipError_t e = c->gated ? hipHostGetDevicePointer(reinterpret_cast<void**>(&dgate), H.gate, 0) : hipErrorOutOfMemory;
      if (e == hipSuccess) {
        hipLaunchKernelGGL(hub_gate_kernel, dim3(1), dim3(64), 0, c->xfer, dgate, uint64_t(H.stall_s * 1.0e8));
        e = hipGetLastError();
      }
      if (e == hipSuccess) e = hipEventRecord(c->gated, c->xfer);
      if (e != hipSuccess) return hip_fail(e, "hdd_comm_post: injected stall (device transport)");
      packed_ev = c->gated;
      H.stall_rank = -1;   // one post
    }
  }
  {   // 1. publish
    std::lock_guard<std::mutex> lk(H.m);
    for (auto& [dst, msgs] : out) {
      auto& q = H.ch[size_t(me) * n + dst];
      q.msgs = msgs;
      q.packed = packed_ev;
      ++q.sent;
    }
  }
  H.cv.notify_all();
  // 2. receives: wait for each source's publication, copy on the transfer stream, record copied
  for (auto& [src, msgs] : in) {
    auto& q = H.ch[size_t(src) * n + me];
    std::vector<std::pair<const double*, int64_t>> sent;
    hipEvent_t packed;
    {
      std::unique_lock<std::mutex> lk(H.m);
      if (!H.cv.wait_for(lk, limit, [&] { return q.sent > q.consumed || !H.failed.empty(); }))
        return fail(lk, "rank " + std::to_string(me) + " timed out waiting for rank " + std::to_string(src));
      if (!H.failed.empty()) return set_error(HDD_ERR_INVALID, "hdd_comm_post (device transport): " + H.failed);
      if (q.msgs.size() != msgs.size())
        return fail(lk, "rank " + std::to_string(src) + " sent " + std::to_string(q.msgs.size()) + " messages to rank " +
                            std::to_string(me) + ", which receives " + std::to_string(msgs.size()));
      for (size_t i = 0; i < msgs.size(); ++i)
        if (q.msgs[i].second != msgs[i].second)
          return fail(lk, "message size mismatch between rank " + std::to_string(src) + " and rank " + std::to_string(me));
      sent = q.msgs;
      packed = q.packed;
    }
    hipError_t e = hipStreamWaitEvent(c->xfer, packed, 0);
    for (size_t i = 0; i < msgs.size() && e == hipSuccess; ++i)
      e = hipMemcpyAsync(msgs[i].first, sent[i].first, size_t(msgs[i].second) * sizeof(double), hipMemcpyDefault, c->xfer);
    if (e == hipSuccess) e = hipEventRecord(c->copied[size_t(src)], c->xfer);
    if (e != hipSuccess) {
      std::unique_lock<std::mutex> lk(H.m);
      return fail(lk, std::string("HIP error on rank ") + std::to_string(me) + ": " + hipGetErrorString(e));
    }
    {
      std::lock_guard<std::mutex> lk(H.m);
      q.copied = c->copied[size_t(src)];
      ++q.consumed;
    }
    H.cv.notify_all();
  }
  // 3. sends complete when every destination has copied them
  for (auto& [dst, msgs] : out) {
    auto& q = H.ch[size_t(me) * n + dst];
    hipEvent_t copied;
    {
      std::unique_lock<std::mutex> lk(H.m);
      if (!H.cv.wait_for(lk, limit, [&] { return q.consumed == q.sent || !H.failed.empty(); }))
        return fail(lk, "rank " + std::to_string(me) + " timed out waiting for rank " + std::to_string(dst) + " to receive");
      if (!H.failed.empty()) return set_error(HDD_ERR_INVALID, "hdd_comm_post (device transport): " + H.failed);
      copied = q.copied;
    }
    const hipError_t e = hipStreamWaitEvent(c->xfer, copied, 0);
    if (e != hipSuccess) return hip_fail(e, "hdd_comm_post: wait for the receivers (device transport)");
  }
  return HDD_OK;
}

// direct (RCCL only; the serial step): the group send/recv on `stream` itself instead of the transfer stream --
// nothing overlaps it there, and it saves the two cross-stream hops (ready -> transfer stream, done -> `stream`),
// ~5 us each on the one-card traces; the ready / done events are still recorded for the watchdog.
// also_ready / also_done (optional): events of the caller recorded right after the communicator's own ready / done
// events on the same streams -- the sharded step's watchdog stages, owned by the shard, so that a later post on the
// same communicator or its destruction cannot change what the step query reports
static int comm_post(hdd_comm* c, int32_t n_peers, const int32_t* peers, const double* const* d_send,
                     const int64_t* send_count, double* const* d_recv, const int64_t* recv_count, void* stream,
                     bool direct, hipEvent_t also_ready = nullptr, hipEvent_t also_done = nullptr)
{
  if (!c || n_peers < 0 || (n_peers && (!peers || !d_send || !send_count || !d_recv || !recv_count)))
    return set_error(HDD_ERR_INVALID, "hdd_comm_post: invalid argument");
  const hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e = hipSetDevice(c->device);
  if (e != hipSuccess) return hip_fail(e, "hdd_comm_post: hipSetDevice");
  c->last_peers.clear();
  for (int32_t k = 0; k < n_peers; ++k)
    if (std::find(c->last_peers.begin(), c->last_peers.end(), peers[k]) == c->last_peers.end())
      c->last_peers.push_back(peers[k]);
  c->direct = nullptr;
  if (direct && (c->kind == hdd_comm::RCCL_OWNED || c->kind == hdd_comm::RCCL_WRAPPED)) {
    e = hipEventRecord(c->ready, s);
    if (e == hipSuccess && also_ready) e = hipEventRecord(also_ready, s);
    if (e != hipSuccess) return hip_fail(e, "hdd_comm_post: record ready");
    const RcclApi& R = rccl();
    ncclResult_t r = R.GroupStart();
    if (r != ncclSuccess) return nccl_fail(r, "ncclGroupStart");
    for (int32_t k = 0; k < n_peers; ++k) {
      if (send_count[k] > 0) {
        r = R.Send(d_send[k], size_t(send_count[k]), ncclFloat64, peers[k], c->nccl, s);
        if (r != ncclSuccess) break;
      }
      if (recv_count[k] > 0) {
        r = R.Recv(d_recv[k], size_t(recv_count[k]), ncclFloat64, peers[k], c->nccl, s);
        if (r != ncclSuccess) break;
      }
    }
    const ncclResult_t r2 = R.GroupEnd();
    if (r != ncclSuccess) return nccl_fail(r, "ncclSend/ncclRecv");
    if (r2 != ncclSuccess) return nccl_fail(r2, "ncclGroupEnd");
    e = hipEventRecord(c->done, s);
    if (e == hipSuccess && also_done) e = hipEventRecord(also_done, s);
    if (e != hipSuccess) return hip_fail(e, "hdd_comm_post: record completion");
    c->posted = true;
    c->direct = s;
    return HDD_OK;
  }
  if (c->kind != hdd_comm::HOST) {
    // the transfer stream starts after the packs already enqueued on `stream`
    e = hipEventRecord(c->ready, s);
    if (e == hipSuccess && also_ready) e = hipEventRecord(also_ready, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(c->xfer, c->ready, 0);
    if (e != hipSuccess) return hip_fail(e, "hdd_comm_post: order transfer after pack");
    if (c->kind == hdd_comm::DEVICE) {
      const int rc = device_post(c, n_peers, peers, d_send, send_count, d_recv, recv_count);
      if (rc) return rc;
      e = hipEventRecord(c->done, c->xfer);
      if (e == hipSuccess && also_done) e = hipEventRecord(also_done, c->xfer);
      if (e != hipSuccess) return hip_fail(e, "hdd_comm_post: record completion");
      c->posted = true;
      return HDD_OK;
    }
    const RcclApi& R = rccl();
    ncclResult_t r = R.GroupStart();
    if (r != ncclSuccess) return nccl_fail(r, "ncclGroupStart");
    for (int32_t k = 0; k < n_peers; ++k) {
      if (send_count[k] > 0) {
        r = R.Send(d_send[k], size_t(send_count[k]), ncclFloat64, peers[k], c->nccl, c->xfer);
        if (r != ncclSuccess) break;
      }
      if (recv_count[k] > 0) {
        r = R.Recv(d_recv[k], size_t(recv_count[k]), ncclFloat64, peers[k], c->nccl, c->xfer);
        if (r != ncclSuccess) break;
      }
    }
    const ncclResult_t r2 = R.GroupEnd();
    if (r != ncclSuccess) return nccl_fail(r, "ncclSend/ncclRecv");
    if (r2 != ncclSuccess) return nccl_fail(r2, "ncclGroupEnd");
    e = hipEventRecord(c->done, c->xfer);
    if (e == hipSuccess && also_done) e = hipEventRecord(also_done, c->xfer);
    if (e != hipSuccess) return hip_fail(e, "hdd_comm_post: record completion");
    c->posted = true;
    return HDD_OK;
  }
  // host-staged: device -> pinned host -> fn -> device, all ordered on `stream`
  size_t total = 0;
  for (int32_t k = 0; k < n_peers; ++k) {
    if (send_count[k] < 0 || recv_count[k] < 0) return set_error(HDD_ERR_INVALID, "hdd_comm_post: negative count");
    total += size_t(send_count[k]) + size_t(recv_count[k]);
  }
  if (total > c->pinned_doubles) {
    if (c->pinned) (void)hipHostFree(c->pinned);
    c->pinned = nullptr;
    c->pinned_doubles = 0;
    e = hipHostMalloc(reinterpret_cast<void**>(&c->pinned), std::max<size_t>(total, 1) * sizeof(double), 0);
    if (e != hipSuccess) return hip_fail(e, "hdd_comm_post: pinned staging");
    c->pinned_doubles = total;
  }
  std::vector<const double*> hs(n_peers);
  std::vector<double*> hr(n_peers);
  size_t off = 0;
  for (int32_t k = 0; k < n_peers; ++k) {
    hs[k] = c->pinned + off;
    off += size_t(send_count[k]);
    hr[k] = c->pinned + off;
    off += size_t(recv_count[k]);
    if (send_count[k]) {
      e = hipMemcpyAsync(const_cast<double*>(hs[k]), d_send[k], size_t(send_count[k]) * sizeof(double),
                         hipMemcpyDeviceToHost, s);
      if (e != hipSuccess) return hip_fail(e, "hdd_comm_post: D2H");
    }
  }
  e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(e, "hdd_comm_post: synchronize");
  const int rc = c->fn(c->user, n_peers, peers, hs.data(), send_count, hr.data(), recv_count);
  if (rc != HDD_OK) return set_error(rc, "hdd_comm_post: host transport failed (status " + std::to_string(rc) + ")");
  for (int32_t k = 0; k < n_peers; ++k)
    if (recv_count[k]) {
      e = hipMemcpyAsync(d_recv[k], hr[k], size_t(recv_count[k]) * sizeof(double), hipMemcpyHostToDevice, s);
      if (e != hipSuccess) return hip_fail(e, "hdd_comm_post: H2D");
    }
  // the staging buffer is reused by the next post: the copies must have left it
  e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(e, "hdd_comm_post: synchronize");
  c->posted = true;
  return HDD_OK;
}

extern "C" int hdd_comm_post(hdd_comm* c, int32_t n_peers, const int32_t* peers, const double* const* d_send,
                             const int64_t* send_count, double* const* d_recv, const int64_t* recv_count, void* stream)
{
  return comm_post(c, n_peers, peers, d_send, send_count, d_recv, recv_count, stream, false);
}

extern "C" int hdd_comm_post_direct(hdd_comm* c, int32_t n_peers, const int32_t* peers, const double* const* d_send,
                                    const int64_t* send_count, double* const* d_recv, const int64_t* recv_count,
                                    void* stream)
{
  return comm_post(c, n_peers, peers, d_send, send_count, d_recv, recv_count, stream, true);
}

extern "C" int hdd_comm_wait(hdd_comm* c, void* stream)
{
  if (!c) return set_error(HDD_ERR_INVALID, "hdd_comm_wait: null comm");
  if (!c->posted) return HDD_OK;
  c->posted = false;
  if (c->kind == hdd_comm::HOST) return HDD_OK;   // already ordered on the stream by hdd_comm_post
  if (c->direct && c->direct == static_cast<hipStream_t>(stream)) {   // posted on this very stream
    c->direct = nullptr;
    return HDD_OK;
  }
  hipError_t e = hipSetDevice(c->device);
  if (e == hipSuccess) e = hipStreamWaitEvent(static_cast<hipStream_t>(stream), c->done, 0);
  return e == hipSuccess ? HDD_OK : hip_fail(e, "hdd_comm_wait");
}

// ------------------------------------------------------------------------------------------------
// shards
// ------------------------------------------------------------------------------------------------
struct hdd_shard {
  int device = 0;
  hdd_local* local = nullptr;
  hdd_grid_info gi{};
  hdd_local_info li{};
  int32_t rank = 0, nranks = 1, s_begin = 0, s_end = 0, degree = 1;
  int64_t nnz = 0;
  std::vector<int64_t> gid;            // host global ids [n_local]
  // device mesh (shard-owned)
  double* d_coords = nullptr;
  int32_t* d_nbrs = nullptr;
  uint32_t* d_finfo = nullptr;
  int64_t* d_gid = nullptr;
  int32_t* d_ev = nullptr;             // vertex-indexed geometry (2d): element -> local vertex ids
  double* d_vxy = nullptr;             //   and the rank-local vertex coordinates (owned + ghost elements')
  // halo
  std::vector<int32_t> peers;
  std::vector<int64_t> send_prefix, recv_prefix, recv_col0;
  int32_t* d_send_idx = nullptr;
  double* d_sbuf = nullptr;
  double* d_rbuf = nullptr;
  int32_t max_rows = 0;
  // tiles
  int32_t* d_tiles_in = nullptr;
  int32_t* d_tiles_bd = nullptr;
  int32_t* d_fix = nullptr;            // owned elements (relative to own_begin) with a ghost face neighbour
  int64_t n_tiles = 0, n_in = 0, n_bd = 0, n_fix = 0;
  int64_t halo_faces = 0;
  // host copies of the plan (hdd_shard_halo_lists / hdd_shard_tile_lists)
  std::vector<int32_t> send_idx, tiles_in, tiles_bd;
  bool host_only = false;          // created without a context: no device arrays
  // side stream of the loopback study (HDD_SHARD_NO_TRANSFER): pack + copies off the assembly stream, as the
  // RCCL path runs them on the transfer stream; created on first use
  hipStream_t aux = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  double* d_fixbuf = nullptr;          // side buffers of the off-stream fixup (n_comp x (n_fix + 1) x fix_rb)
  size_t fixbuf_doubles = 0;
  // watchdog (hdd_block_step_query / _sync): the stages the last step recorded events for, and a marker event
  uint32_t stages = 0;                 // bit 0: pack (ev_pack), 1: exchange (ev_xdone), 2: element pass (ev_out)
  hipEvent_t ev_pack = nullptr, ev_xdone = nullptr;   // recorded beside the communicator's ready / done (comm_post)
  std::vector<int32_t> stage_peers;    // the halo peers of the last step (watchdog messages)
  hipEvent_t ev_mark = nullptr;
  bool marked = false;
};

extern "C" void hdd_shard_destroy(hdd_shard* sh)
{
  if (!sh) return;
  if (!sh->host_only) (void)hipSetDevice(sh->device);
  if (sh->aux) (void)hipStreamDestroy(sh->aux);
  if (sh->ev_in) (void)hipEventDestroy(sh->ev_in);
  if (sh->ev_out) (void)hipEventDestroy(sh->ev_out);
  if (sh->ev_mark) (void)hipEventDestroy(sh->ev_mark);
  if (sh->ev_pack) (void)hipEventDestroy(sh->ev_pack);
  if (sh->ev_xdone) (void)hipEventDestroy(sh->ev_xdone);
  for (void* p : {static_cast<void*>(sh->d_coords), static_cast<void*>(sh->d_nbrs), static_cast<void*>(sh->d_finfo),
                  static_cast<void*>(sh->d_gid), static_cast<void*>(sh->d_send_idx), static_cast<void*>(sh->d_sbuf),
                  static_cast<void*>(sh->d_rbuf), static_cast<void*>(sh->d_tiles_in),
                  static_cast<void*>(sh->d_tiles_bd), static_cast<void*>(sh->d_ev), static_cast<void*>(sh->d_vxy),
                  static_cast<void*>(sh->d_fix), static_cast<void*>(sh->d_fixbuf)})
    if (p) (void)hipFree(p);
  if (sh->local) hdd_local_destroy(sh->local);
  delete sh;
}

extern "C" int hdd_shard_create(hdd_ctx* ctx, const hdd_grid* g, int32_t nranks, int32_t rank, const int32_t* owner,
                                hdd_shard** out)
{
  if (!g || !out || nranks < 1 || rank < 0 || rank >= nranks)
    return set_error(HDD_ERR_INVALID, "hdd_shard_create: invalid argument");
  hdd_grid_info gi{};
  int rc = hdd_grid_get_info(g, &gi);
  if (rc) return rc;
  std::vector<int32_t> own(size_t(gi.n_subdomains));
  if (owner) {
    std::copy(owner, owner + gi.n_subdomains, own.begin());
  } else {
    if (nranks > gi.n_subdomains)
      return set_error(HDD_ERR_INVALID, "hdd_shard_create: more ranks than subdomains");
    for (int32_t r = 0; r < nranks; ++r)
      for (int64_t s = int64_t(r) * gi.n_subdomains / nranks; s < int64_t(r + 1) * gi.n_subdomains / nranks; ++s)
        own[size_t(s)] = r;
  }
  int32_t s0 = -1, s1 = -1;
  for (int32_t s = 0; s < gi.n_subdomains; ++s) {
    if (own[s] < 0 || own[s] >= nranks) return set_error(HDD_ERR_RANGE, "hdd_shard_create: owner out of range");
    if (own[s] != rank) continue;
    if (s0 < 0) s0 = s;
    else if (s1 != s) return set_error(HDD_ERR_UNSUPPORTED, "hdd_shard_create: owned subdomains must be contiguous");
    s1 = s + 1;
  }
  if (s0 < 0) return set_error(HDD_ERR_INVALID, "hdd_shard_create: rank owns no subdomain");

  auto* sh = new hdd_shard;
  auto fail = [&](int code) {
    hdd_shard_destroy(sh);
    return code;
  };
  sh->device = hdd::ctx_device(ctx);
  sh->host_only = !ctx;
  sh->gi = gi;
  sh->rank = rank;
  sh->nranks = nranks;
  sh->s_begin = s0;
  sh->s_end = s1;
  if (gi.elem_type == HDD_HEX)
    while ((sh->degree + 1) * (sh->degree + 1) * (sh->degree + 1) < gi.nb) ++sh->degree;
  rc = hdd_local_create(g, s0, s1, &sh->local);
  if (rc) return fail(rc);
  rc = hdd_local_get_info(sh->local, &sh->li);
  if (rc) return fail(rc);
  const int64_t nl = sh->li.n_local, ob = sh->li.own_begin, oe = sh->li.own_end;
  std::vector<double> coords(size_t(gi.dim) * gi.nvpe * nl);
  std::vector<int32_t> nbrs(size_t(gi.nfaces) * nl);
  std::vector<uint32_t> finfo(static_cast<size_t>(nl));
  sh->gid.resize(size_t(nl));
  rc = hdd_local_fill(sh->local, coords.data(), nbrs.data(), finfo.data(), sh->gid.data(), nullptr);
  if (rc) return fail(rc);
  rc = hdd_dg_pattern_count(gi.nfaces, gi.nb, nl, ob, oe, nbrs.data(), &sh->nnz);
  if (rc) return fail(rc);
  // vertex-indexed geometry of the local elements (2d): what the P1 / Q1 kernels read
  std::vector<int32_t> ev;
  std::vector<double> vxy;
  if (gi.dim == 2) {
    int64_t nvl = 0;
    rc = hdd_local_vertices(sh->local, &nvl, nullptr, nullptr);
    if (rc) return fail(rc);
    ev.resize(size_t(gi.nvpe) * nl);
    vxy.resize(size_t(2) * nvl);
    rc = hdd_local_vertices(sh->local, &nvl, ev.data(), vxy.data());
    if (rc) return fail(rc);
  }

  // halo plan: peers ascending, send lists concatenated in peer order
  int32_t np = 0;
  rc = hdd_local_halo_plan(sh->local, own.data(), rank, &np, nullptr, nullptr, nullptr, nullptr);
  if (rc) return fail(rc);
  if (np > SH_MAX_PEERS) return fail(set_error(HDD_ERR_UNSUPPORTED, "hdd_shard_create: more than 64 halo peers"));
  sh->peers.resize(size_t(np));
  std::vector<int64_t> sc(static_cast<size_t>(np)), ro(static_cast<size_t>(np)), rcnt(static_cast<size_t>(np));
  rc = hdd_local_halo_plan(sh->local, own.data(), rank, &np, sh->peers.data(), sc.data(), ro.data(), rcnt.data());
  if (rc) return fail(rc);
  sh->send_prefix.assign(size_t(np) + 1, 0);
  sh->recv_prefix.assign(size_t(np) + 1, 0);
  sh->recv_col0 = ro;
  for (int32_t k = 0; k < np; ++k) {
    sh->send_prefix[k + 1] = sh->send_prefix[k] + sc[k];
    sh->recv_prefix[k + 1] = sh->recv_prefix[k] + rcnt[k];
  }
  std::vector<int32_t> send_idx(size_t(sh->send_prefix[np]));
  for (int32_t k = 0; k < np; ++k) {
    if (!sc[k]) continue;
    rc = hdd_local_send_list(sh->local, own.data(), rank, k, send_idx.data() + sh->send_prefix[k]);
    if (rc) return fail(rc);
  }

  // interior / halo-boundary tiles (64 owned elements; a boundary tile has an element with a ghost face)
  const int64_t n_own = oe - ob;
  sh->n_tiles = (n_own + 63) / 64;
  std::vector<int32_t> tin, tbd, fix;
  for (int64_t t = 0; t < sh->n_tiles; ++t) {
    bool ghost = false;
    for (int64_t e = ob + 64 * t; e < std::min(oe, ob + 64 * t + 64); ++e) {
      bool eg = false;
      for (int f = 0; f < gi.nfaces; ++f) {
        const int32_t n = nbrs[size_t(f) * nl + e];
        if (n >= 0 && (n < ob || n >= oe)) {
          eg = true;
          ++sh->halo_faces;
        }
      }
      if (eg) fix.push_back(int32_t(e - ob));
      ghost |= eg;
    }
    (ghost ? tbd : tin).push_back(int32_t(t));
  }
  sh->n_fix = int64_t(fix.size());
  sh->n_in = int64_t(tin.size());
  sh->n_bd = int64_t(tbd.size());
  sh->send_idx = send_idx;
  sh->tiles_in = tin;
  sh->tiles_bd = tbd;
  // message rows: coordinates + symmetric tensor + one row per diffusion-factor component
  sh->max_rows = gi.dim * gi.nvpe + (gi.dim == 3 ? 6 : 3) + HDD_MAX_COMP;
  if (!ctx) {   // host-only shard: plan and local mesh, nothing on a device (CPU tests of the halo protocol)
    sh->host_only = true;
    *out = sh;
    return HDD_OK;
  }

  hipError_t e = hipSetDevice(sh->device);
  if (e == hipSuccess) e = upload(&sh->d_coords, coords);
  if (e == hipSuccess) e = upload(&sh->d_nbrs, nbrs);
  if (e == hipSuccess) e = upload(&sh->d_finfo, finfo);
  if (e == hipSuccess) e = upload(&sh->d_gid, sh->gid);
  if (e == hipSuccess && !ev.empty()) e = upload(&sh->d_ev, ev);
  if (e == hipSuccess && !vxy.empty()) e = upload(&sh->d_vxy, vxy);
  if (e == hipSuccess) e = upload(&sh->d_send_idx, send_idx);
  if (e == hipSuccess) e = upload(&sh->d_tiles_in, tin);
  if (e == hipSuccess) e = upload(&sh->d_tiles_bd, tbd);
  if (e == hipSuccess) e = upload(&sh->d_fix, fix);
  if (e == hipSuccess && sh->send_prefix[np])
    e = hipMalloc(&sh->d_sbuf, size_t(sh->max_rows) * sh->send_prefix[np] * sizeof(double));
  if (e == hipSuccess && sh->recv_prefix[np])
    e = hipMalloc(&sh->d_rbuf, size_t(sh->max_rows) * sh->recv_prefix[np] * sizeof(double));
  if (e != hipSuccess) return fail(hip_fail(e, "hdd_shard_create: upload"));
  *out = sh;
  return HDD_OK;
}

extern "C" int hdd_shard_get_info(const hdd_shard* sh, hdd_shard_info* o)
{
  if (!sh || !o) return set_error(HDD_ERR_INVALID, "hdd_shard_get_info: null argument");
  o->n_local = sh->li.n_local;
  o->own_begin = sh->li.own_begin;
  o->own_end = sh->li.own_end;
  o->n_ghost = sh->li.n_ghost;
  o->global_first = sh->li.global_first;
  o->n_rows = int64_t(sh->gi.nb) * (sh->li.own_end - sh->li.own_begin);
  o->n_cols = int64_t(sh->gi.nb) * sh->gi.n_elements;
  o->nnz = sh->nnz;
  o->rank = sh->rank;
  o->nranks = sh->nranks;
  o->s_begin = sh->s_begin;
  o->s_end = sh->s_end;
  o->n_peers = int32_t(sh->peers.size());
  o->nb = sh->gi.nb;
  o->n_tiles = sh->n_tiles;
  o->n_tiles_interior = sh->n_in;
  o->n_tiles_boundary = sh->n_bd;
  o->halo_send = sh->send_prefix.back();
  o->halo_recv = sh->recv_prefix.back();
  o->halo_faces = sh->halo_faces;
  o->halo_elements = sh->n_fix;
  return HDD_OK;
}

extern "C" int hdd_shard_halo_lists(const hdd_shard* sh, int32_t* peers, int64_t* send_prefix, int32_t* send_idx,
                                    int64_t* recv_prefix, int64_t* recv_col0)
{
  if (!sh) return set_error(HDD_ERR_INVALID, "hdd_shard_halo_lists: null shard");
  const size_t np = sh->peers.size();
  if (peers) std::copy(sh->peers.begin(), sh->peers.end(), peers);
  if (send_prefix) std::copy(sh->send_prefix.begin(), sh->send_prefix.end(), send_prefix);
  if (send_idx) std::copy(sh->send_idx.begin(), sh->send_idx.end(), send_idx);
  if (recv_prefix) std::copy(sh->recv_prefix.begin(), sh->recv_prefix.end(), recv_prefix);
  if (recv_col0) std::copy(sh->recv_col0.begin(), sh->recv_col0.begin() + np, recv_col0);
  return HDD_OK;
}

extern "C" int hdd_shard_tile_lists(const hdd_shard* sh, int32_t* interior, int32_t* boundary)
{
  if (!sh) return set_error(HDD_ERR_INVALID, "hdd_shard_tile_lists: null shard");
  if (interior) std::copy(sh->tiles_in.begin(), sh->tiles_in.end(), interior);
  if (boundary) std::copy(sh->tiles_bd.begin(), sh->tiles_bd.end(), boundary);
  return HDD_OK;
}

extern "C" int hdd_shard_mesh(const hdd_shard* sh, hdd_mesh* m)
{
  if (!sh || !m) return set_error(HDD_ERR_INVALID, "hdd_shard_mesh: null argument");
  if (sh->host_only) return set_error(HDD_ERR_INVALID, "hdd_shard_mesh: host-only shard (no device mesh)");
  *m = hdd_mesh{sh->gi.elem_type, sh->gi.elem_type == HDD_HEX ? sh->degree : 1, sh->li.n_local, sh->li.own_begin,
                sh->li.own_end, sh->d_coords, sh->d_nbrs, sh->d_finfo, sh->d_ev, sh->d_vxy};
  return HDD_OK;
}

extern "C" int hdd_shard_global_ids(const hdd_shard* sh, int64_t* global_id)
{
  if (!sh || !global_id) return set_error(HDD_ERR_INVALID, "hdd_shard_global_ids: null argument");
  std::copy(sh->gid.begin(), sh->gid.end(), global_id);
  return HDD_OK;
}

extern "C" int hdd_shard_centers(const hdd_shard* sh, double* centers)
{
  if (!sh || !centers) return set_error(HDD_ERR_INVALID, "hdd_shard_centers: null argument");
  return hdd_local_centers(sh->local, centers);
}

extern "C" int hdd_shard_pattern_fill(hdd_ctx* ctx, const hdd_shard* sh, int64_t* d_row_ptr, int32_t* d_col,
                                      int64_t* d_elem_ptr, void* stream)
{
  if (!ctx || !sh || !d_row_ptr || !d_col || !d_elem_ptr)
    return set_error(HDD_ERR_INVALID, "hdd_shard_pattern_fill: null argument");
  if (sh->host_only) return set_error(HDD_ERR_INVALID, "hdd_shard_pattern_fill: host-only shard (created without a context)");
  hdd_mesh m;
  hdd_shard_mesh(sh, &m);
  int64_t nnz = 0;
  int rc = hdd_pattern_elem_ptr_device(ctx, &m, sh->gi.nb, d_elem_ptr, &nnz, stream);
  if (rc) return rc;
  if (nnz != sh->nnz) return set_error(HDD_ERR_INVALID, "hdd_shard_pattern_fill: nnz mismatch (internal)");
  rc = hdd_pattern_fill_device(ctx, &m, sh->gi.nb, sh->d_gid, d_elem_ptr, d_row_ptr, d_col, stream);
  if (rc) return rc;
  const hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
  return e == hipSuccess ? HDD_OK : hip_fail(e, "hdd_shard_pattern_fill: synchronize");
}

static hipError_t launch_halo(bool pack, const HaloArgs& a, hipStream_t s)
{
  const int64_t total = int64_t(a.row_first[a.n_arrays]) * a.prefix[a.n_peers];
  if (total == 0) return hipSuccess;
  const unsigned grid = unsigned(std::min<int64_t>((total + 255) / 256, 1024));
  if (pack) hipLaunchKernelGGL(halo_pack_kernel, dim3(grid), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(halo_unpack_kernel, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

extern "C" int hdd_block_assemble_sharded(hdd_ctx* ctx, hdd_shard* sh, hdd_comm* comm, const hdd_scalar_fn* kappa,
                                          int32_t n_comp, const hdd_tensor_fn* tensor,
                                          const hdd_swipdg_params* params, const hdd_csr* pattern,
                                          double* const* d_vals, uint32_t flags, void* stream)
{
  if (!ctx || !sh || !kappa || !tensor || !params || !pattern || !d_vals)
    return set_error(HDD_ERR_INVALID, "hdd_block_assemble_sharded: null argument");
  if (sh->host_only)
    return set_error(HDD_ERR_INVALID, "hdd_block_assemble_sharded: host-only shard (created without a context)");
  if (n_comp < 1 || n_comp > HDD_MAX_COMP)
    return set_error(HDD_ERR_INVALID, "hdd_block_assemble_sharded: need 1 <= n_comp <= HDD_MAX_COMP");
  if (pattern->nnz != sh->nnz || pattern->n_rows != int64_t(sh->gi.nb) * (sh->li.own_end - sh->li.own_begin))
    return set_error(HDD_ERR_INVALID, "hdd_block_assemble_sharded: pattern does not belong to this shard");
  hdd_mesh m;
  hdd_shard_mesh(sh, &m);
  if (flags & HDD_SHARD_HALO_GEOMETRY) {   // ghost geometry arrives through the halo: element-major coords
    m.elem_vertices = nullptr;
    m.vertex_coords = nullptr;
  }
  const hipStream_t s = static_cast<hipStream_t>(stream);

  // halo rows: [coordinates] [tensor] [per-element diffusion factors (each distinct array once)]
  HaloArgs h{};
  h.ld = sh->li.n_local;
  h.n_peers = int32_t(sh->peers.size());
  // (no de-duplication of arrays passed twice: the message layout must depend on the kinds only, which
  // every rank passes alike, never on pointer identity)
  auto add = [&](double* p, int rows) {
    h.arr[h.n_arrays] = p;
    h.row_first[h.n_arrays + 1] = h.row_first[h.n_arrays] + rows;
    ++h.n_arrays;
  };
  if (flags & HDD_SHARD_HALO_GEOMETRY) add(sh->d_coords, sh->gi.dim * sh->gi.nvpe);
  if (tensor->kind == HDD_TENSOR_ISO_PER_ELEM || tensor->kind == HDD_TENSOR_SYM_PER_ELEM) {
    if (!tensor->per_elem) return set_error(HDD_ERR_INVALID, "hdd_block_assemble_sharded: tensor per_elem missing");
    add(const_cast<double*>(tensor->per_elem),
        tensor->kind == HDD_TENSOR_ISO_PER_ELEM ? 1 : (sh->gi.dim == 3 ? 6 : 3));
  }
  for (int32_t c = 0; c < n_comp; ++c)
    if (kappa[c].kind == HDD_FN_PER_ELEM) {
      if (!kappa[c].per_elem) return set_error(HDD_ERR_INVALID, "hdd_block_assemble_sharded: kappa per_elem missing");
      add(const_cast<double*>(kappa[c].per_elem), 1);
    }
  const bool exchange = h.n_peers > 0 && !(flags & HDD_SHARD_NO_HALO) && h.n_arrays > 0;
  if (!exchange) return hdd_swipdg_assemble(ctx, &m, kappa, n_comp, tensor, params, pattern, d_vals, stream);
  const bool transfer = !(flags & HDD_SHARD_NO_TRANSFER);
  if (!comm && transfer)
    return set_error(HDD_ERR_INVALID, "hdd_block_assemble_sharded: the shard has halo peers but comm is NULL");
  const int32_t R = h.row_first[h.n_arrays];
  if (R > sh->max_rows) return set_error(HDD_ERR_INVALID, "hdd_block_assemble_sharded: too many halo rows");

  hipError_t e = hipSetDevice(sh->device);
  if (e != hipSuccess) return hip_fail(e, "hdd_block_assemble_sharded: hipSetDevice");
  sh->stages = 0;
  sh->marked = false;
  // Default schedule by element type and peer count (one-card step study, profiles/r04/e_reserve/): P1 ranks with
  // two peers split the tiles -- interior tiles during the exchange, the 2 % of tiles with a ghost-adjacent element
  // after it (C2 N = 8 middle rank +0.8 / +4.0 % over one launch, against +10.1 % for the side-buffer fixup and
  // +26.5 % in place, whose row blocks share cache lines with the tiles' stores: P1 blocks are 288 B); every other
  // shard keeps the off-stream element fixup in place (Q1: its split costs +18 %).
  const bool default_schedule = !(flags & (HDD_SHARD_FIX_INLINE | HDD_SHARD_FIX_SCATTER | HDD_SHARD_FIX_INPLACE));
  const bool split = (flags & HDD_SHARD_SPLIT_TILES) != 0 ||
                     (default_schedule && sh->gi.elem_type == HDD_SIMPLEX && sh->peers.size() >= 2 && sh->n_in > 0);
  //
  // Round 5, Q1: the serial step by default (pack, exchange, then one half-image launch over every tile).  One-card
  // study on the final kernels (profiles/r05/d_shard/, loopback transfer, back-to-back steps): C4 N = 8 end / middle
  // rank serial +8.5 / +12.3 % over one launch, the overlapped in-place step +16.7 / +20.8 %, the side buffer after
  // the join +13.4 / +18.9 %; N = 2 serial +2.2 / +3.1 %, overlapped +4.3 / +5.0 %.  The kernel trace shows why: the
  // half-image launch holds every wave slot it can (two waves per SIMD, all of the LDS), so the halo kernels beside
  // it wait for the reserved slots (a D2D copy 39 us instead of 5), and each cross-stream join costs ~5 us on the
  // step's critical path.  The overlapped schedules stay selectable (HDD_SHARD_FIX_INPLACE / _FIX_SCATTER / _SPLIT).
  const bool q1_serial = sh->gi.elem_type == HDD_CUBE && default_schedule && !(flags & HDD_SHARD_SPLIT_TILES);
  bool overlap = !(flags & HDD_SHARD_NO_OVERLAP) && sh->gi.elem_type != HDD_HEX && !q1_serial &&
                 (split ? sh->n_in > 0 : true);
  // The pack and the transfer leave the assembly stream when the assembly overlaps them: the RCCL transfer
  // stream (or, in the loopback study, the shard's side stream) waits for the inputs, packs and sends while
  // `stream` starts the assembly at once -- the pack launch is off the critical path.  (The host transport
  // stages through the host on `stream` anyway.)
  hipStream_t ps = s;
  // With the in-place fixup the full-range skip launch is enqueued BEFORE the halo work by default, so it starts at
  // once instead of after the host has issued pack, exchange and element pass (one-card kernel timeline,
  // profiles/r04/n_first/: C4 N = 8 step 113-120 -> 77-79 us when steps do not overlap; back-to-back steps, where the
  // host runs ahead, are unchanged).  HDD_SHARD_LAUNCH_LAST: round 3's order.  The split keeps its pack on `stream`
  // before the interior tiles: packing on the side stream beside them measured +10.0 % against +5.3 % (C2 N = 8
  // middle rank, back-to-back, profiles/r04/o_final/).
#ifdef HDD_ABLATION
  const bool last = (flags & HDD_SHARD_LAUNCH_LAST) != 0;
#else
  const bool last = false;   // (HDD_SHARD_LAUNCH_LAST: ablation builds only)
#endif
  const bool side = overlap && !split;
  if (side) {
    if (transfer && comm->kind != hdd_comm::HOST) {
      ps = comm->xfer;
    } else {   // loopback study, host transport (which stages through the host on this stream)
      if (!sh->aux) {
        e = hipStreamCreateWithFlags(&sh->aux, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&sh->ev_in, local_event_flags());
        if (e == hipSuccess) e = hipEventCreateWithFlags(&sh->ev_out, local_event_flags());
        if (e != hipSuccess) return hip_fail(e, "hdd_block_assemble_sharded: side stream");
      }
      ps = sh->aux;
    }
    if (!sh->ev_in) {
      e = hipEventCreateWithFlags(&sh->ev_in, local_event_flags());
      if (e != hipSuccess) return hip_fail(e, "hdd_block_assemble_sharded: event");
    }
    if (!sh->ev_out) {
      e = hipEventCreateWithFlags(&sh->ev_out, local_event_flags());
      if (e != hipSuccess) return hip_fail(e, "hdd_block_assemble_sharded: event");
    }
  }
  const bool q1 = sh->gi.elem_type == HDD_CUBE;
  // Q1: the pack runs on `stream` ahead of the tile launch.  Issued on the side stream beside the tile launch it
  // waited for a free wave slot: the half-image SKIP kernel holds 256 VGPRs in each of its two waves per SIMD and
  // all of the LDS, so a kernel beside it gets only the reserved workgroup slots -- the pack took 45 us there
  // against 5 us alone, and the element pass behind it ended after the tiles (one-card kernel trace,
  // profiles/r05/d_shard/).  On `stream` it costs its own few microseconds once, ahead of the launch.
  const bool pack_first = side && q1;
  for (int k = 0; k <= h.n_peers; ++k) h.prefix[k] = sh->send_prefix[k];
  h.idx = sh->d_send_idx;
  h.buf = sh->d_sbuf;
  if (pack_first) {
    e = launch_halo(true, h, s);
    if (e != hipSuccess) return hip_fail(e, "hdd_block_assemble_sharded: pack");
  }
  if (side) {
    e = hipEventRecord(sh->ev_in, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(ps, sh->ev_in, 0);
    if (e != hipSuccess) return hip_fail(e, "hdd_block_assemble_sharded: order pack after inputs");
  }
  const bool offfix = side && !split && !(flags & HDD_SHARD_FIX_INLINE) && sh->n_fix > 0;
  // where the fixup writes: in place beside a tile launch that skips those row blocks, or a side buffer + one
  // copy kernel after the join.  Default from the one-card step study (profiles/r03/shard_step/final/, N = 2 and
  // 8): in place, except P1 ranks with two peers (C2 middle ranks: +10 % with the side buffer vs +14 % in place,
  // the P1 tiles' two waves per SIMD leaving the element pass no registers beside them; end ranks +4 % in place
  // vs +8 %); Q1 in place everywhere (+9 % middle / +15 % end rank at N = 8 vs +20 / +13 %)
  //
  // Round 5: Q1 keeps the in-place pass, now beside the half-image kernel's SKIP launch (full SKIP tiles stay on the
  // rotated image and drop the skipped elements' chunks at the store), with the pack ahead of the launch (above).
  // HDD_SHARD_FIX_SCATTER on Q1: the tile launch writes every row block (no SKIP), the ghost-adjacent elements go
  // into a value-major (SoA) side buffer -- each store instruction 64 consecutive doubles -- and one wave per
  // element writes its row block into place after the join (a kernel after the tiles: +18 % at C4 N = 8).
  const bool scatter = offfix && !(flags & HDD_SHARD_FIX_INPLACE) && (flags & HDD_SHARD_FIX_SCATTER);
  // the value-major pass exists for the closed-form Q1 policy only (piecewise-constant kappa: Q1PwcPolicy::emit); a
  // smooth kappa (GenericPolicy) takes the row-block side buffer + hdd_scatter_fix like P1
  bool pwc_kappa = true;
  for (int32_t c = 0; c < n_comp; ++c)
    pwc_kappa = pwc_kappa && (kappa[c].kind == HDD_FN_CONST || kappa[c].kind == HDD_FN_PER_ELEM);
  const bool soa = scatter && q1 && pwc_kappa;
  const int32_t rb = hdd_fix_rb(sh->gi.elem_type);
  const int64_t soa_ld = (sh->n_fix + 1 + 63) & ~int64_t(63);   // SoA rows start 512-byte aligned
  std::vector<double*> fbufs;
  if (scatter) {
    const size_t slot = soa ? size_t(soa_ld) * size_t(rb) : size_t(sh->n_fix + 1) * size_t(rb);
    const size_t need = slot * size_t(n_comp);
    if (need > sh->fixbuf_doubles) {   // first step (or more components): grow; warm up before graph capture
      if (sh->d_fixbuf) (void)hipFree(sh->d_fixbuf);
      sh->d_fixbuf = nullptr;
      sh->fixbuf_doubles = 0;
      e = hipMalloc(reinterpret_cast<void**>(&sh->d_fixbuf), need * sizeof(double));
      if (e != hipSuccess) return hip_fail(e, "hdd_block_assemble_sharded: fixup buffer");
      sh->fixbuf_doubles = need;
    }
    for (int32_t c = 0; c < n_comp; ++c) fbufs.push_back(sh->d_fixbuf + size_t(c) * slot);
  }
  // 0. The skip launch first (see above): it needs nothing the exchange delivers (the row blocks that read a ghost
  // column are the element pass's), and the inputs event was recorded above, so the pack does not wait for it.
  const int32_t reserve = int32_t(std::min<int64_t>((sh->n_fix + 63) / 64, 256));
  bool first = false;
  if (!last && offfix && (!scatter || soa)) {
    const int rc0 = soa ? hdd_assemble_reserve(ctx, &m, kappa, n_comp, tensor, params, pattern, d_vals, stream, reserve)
                        : hdd_assemble_skip_ghost(ctx, &m, kappa, n_comp, tensor, params, pattern, d_vals, stream, reserve);
    if (rc0 == HDD_OK) first = true;
    else if (rc0 != HDD_ERR_UNSUPPORTED) return rc0;   // (unsupported rules: the order below)
  }
  // 1. pack the records the peers need (one launch for every peer; Q1: done above)
  if (!pack_first) {
    e = launch_halo(true, h, ps);
    if (e != hipSuccess) return hip_fail(e, "hdd_block_assemble_sharded: pack");
  }
  // 2. post the exchange.  The receives land straight in the ghost columns: the ghosts of one owner are
  // contiguous (recv_col0), so peer k's message is R row messages [row r][count_k], each received into
  // arr(r)[row(r) ld + recv_col0[k] ...] -- no receive buffer, no unpack launch.  Sender and receiver list the
  // rows in the same order (the layout depends on the kinds only), which is how RCCL / the host transports
  // match repeated (peer) messages.
  int rc = HDD_OK;
  double* loop_buf = sh->d_rbuf;   // what the loopback's unpack reads
  if (transfer) {
    std::vector<int32_t> mp;
    std::vector<const double*> ms;
    std::vector<double*> mr;
    std::vector<int64_t> mn, mrn;
    for (int k = 0; k < h.n_peers; ++k) {
      const int64_t scnt = sh->send_prefix[k + 1] - sh->send_prefix[k];
      const int64_t rcnt = sh->recv_prefix[k + 1] - sh->recv_prefix[k];
      for (int32_t r = 0, a = 0; r < R; ++r) {
        while (a + 1 < h.n_arrays && h.row_first[a + 1] <= r) ++a;
        mp.push_back(sh->peers[size_t(k)]);
        ms.push_back(sh->d_sbuf + int64_t(R) * sh->send_prefix[k] + int64_t(r) * scnt);
        mn.push_back(scnt);
        mr.push_back(h.arr[a] + int64_t(r - h.row_first[a]) * h.ld + sh->recv_col0[k]);
        mrn.push_back(rcnt);
      }
    }
    // serial step (no overlap, ps == s): RCCL runs straight on `stream`
    const bool staged = comm->kind != hdd_comm::HOST;
    if (staged && !sh->ev_pack && hipEventCreateWithFlags(&sh->ev_pack, hipEventDisableTiming) != hipSuccess)
      return set_error(HDD_ERR_HIP, "hdd_block_assemble_sharded: stage event");
    if (staged && !sh->ev_xdone && hipEventCreateWithFlags(&sh->ev_xdone, hipEventDisableTiming) != hipSuccess)
      return set_error(HDD_ERR_HIP, "hdd_block_assemble_sharded: stage event");
    rc = comm_post(comm, int32_t(mp.size()), mp.data(), ms.data(), mn.data(), mr.data(), mrn.data(), ps, !overlap,
                   staged ? sh->ev_pack : nullptr, staged ? sh->ev_xdone : nullptr);
    if (rc == HDD_OK && staged) sh->stages |= 3u;
    if (rc == HDD_OK) sh->stage_peers = comm->last_peers;
    // host transport on the side stream, fixup on `stream`: the ghost columns were written on ps
    if (rc == HDD_OK && side && !offfix && ps != s && comm->kind == hdd_comm::HOST &&
        hipEventRecord(sh->ev_out, ps) != hipSuccess)
      rc = set_error(HDD_ERR_HIP, "hdd_block_assemble_sharded: host transport event");
  } else {   // timing studies: the receive buffers get this rank's own messages (stream-ordered device copies)
    // With equal send and receive counts per peer (every halo here: ghost layers are symmetric) the loopback is ONE
    // kernel, the unpack reading the send buffer -- as the transfer is: RCCL's group kernel receives straight into
    // the ghost columns.  (Round 4 and earlier: a copy per peer + the unpack, i.e. 2-3 kernels for one transfer.)
    bool same = true;
    for (int k = 0; k < h.n_peers; ++k)
      same = same && sh->send_prefix[k + 1] - sh->send_prefix[k] == sh->recv_prefix[k + 1] - sh->recv_prefix[k];
    if (same) loop_buf = sh->d_sbuf;
    std::vector<const double*> sp(size_t(h.n_peers));
    std::vector<double*> rp(size_t(h.n_peers));
    std::vector<int64_t> sn(size_t(h.n_peers)), rn(size_t(h.n_peers));
    for (int k = 0; k < h.n_peers; ++k) {
      sp[k] = sh->d_sbuf + int64_t(R) * sh->send_prefix[k];
      sn[k] = int64_t(R) * (sh->send_prefix[k + 1] - sh->send_prefix[k]);
      rp[k] = sh->d_rbuf + int64_t(R) * sh->recv_prefix[k];
      rn[k] = int64_t(R) * (sh->recv_prefix[k + 1] - sh->recv_prefix[k]);
    }
    for (int k = 0; k < h.n_peers && rc == HDD_OK && !same; ++k) {
      const int64_t n = std::min(sn[k], rn[k]);
      if (n > 0 && hipMemcpyAsync(rp[k], sp[k], size_t(n) * sizeof(double), hipMemcpyDeviceToDevice, ps) != hipSuccess)
        rc = set_error(HDD_ERR_HIP, "hdd_block_assemble_sharded: loopback copy");
    }
    if (rc == HDD_OK && ps != s && hipEventRecord(sh->ev_out, ps) != hipSuccess)
      rc = set_error(HDD_ERR_HIP, "hdd_block_assemble_sharded: loopback event");
  }
  if (rc) return rc;
  // 2b. off-stream fixup (default with a side stream): on the stream the halo lands on, right after it, the
  // ghost-adjacent elements into the side buffer -- concurrent with the assembly below, which needs the LDS this
  // pass does without; the loopback study unpacks there first
  bool fix_pending = false, fix_unsupported = false;
  if (offfix) {
    if (!transfer) {
      for (int k = 0; k <= h.n_peers; ++k) h.prefix[k] = sh->recv_prefix[k];
      for (int k = 0; k < h.n_peers; ++k) h.col0[k] = sh->recv_col0[k];
      h.idx = nullptr;
      h.buf = loop_buf;
      e = launch_halo(false, h, ps);
      if (e != hipSuccess) return hip_fail(e, "hdd_block_assemble_sharded: unpack");
    }
    rc = soa       ? hdd_assemble_elements_soa(ctx, &m, kappa, n_comp, tensor, params, pattern, fbufs.data(), soa_ld,
                                                 sh->d_fix, sh->n_fix, ps)
         : scatter ? hdd_assemble_elements_buf(ctx, &m, kappa, n_comp, tensor, params, pattern, fbufs.data(), sh->d_fix,
                                             sh->n_fix, ps)
                 : hdd_assemble_elements_inplace(ctx, &m, kappa, n_comp, tensor, params, pattern, d_vals, sh->d_fix,
                                                 sh->n_fix, ps);
    if (rc == HDD_ERR_UNSUPPORTED) fix_unsupported = true;   // no list kernel for these rules: range again below
    else if (rc) {
      if (transfer) (void)hdd_comm_wait(comm, stream);
      return rc;
    }
    e = hipEventRecord(sh->ev_out, ps);
    if (e != hipSuccess) return hip_fail(e, "hdd_block_assemble_sharded: record fixup");
    fix_pending = true;
    sh->stages |= 4u;
  }
  // 3. the assembly overlaps the transfer.  Default: EVERY tile (one full-size launch at full rate; the row
  // blocks of the ghost-adjacent elements read ghost columns the receives are still writing and are recomputed
  // in 5).  HDD_SHARD_SPLIT_TILES: the interior tiles only (the kernels that take lists: P1 / Q1 persistent
  // policies) -- a second launch of whole boundary tiles later, which on thin strips is a large fraction.
  if (overlap && !first) {
    // in-place fixup running: the tiles leave the ghost-adjacent elements' row blocks to it
    const bool skip = fix_pending && !scatter && !fix_unsupported;
    rc = split ? hdd_swipdg_assemble_tiles(ctx, &m, kappa, n_comp, tensor, params, pattern, d_vals, sh->d_tiles_in,
                                           sh->n_in, stream)
         : skip ? hdd_assemble_skip_ghost(ctx, &m, kappa, n_comp, tensor, params, pattern, d_vals, stream, reserve)
                : hdd_swipdg_assemble(ctx, &m, kappa, n_comp, tensor, params, pattern, d_vals, stream);
    if (rc == HDD_ERR_UNSUPPORTED && split) overlap = false;   // no tile-list kernel: everything after the halo
    else if (rc) {
      if (transfer) (void)hdd_comm_wait(comm, stream);
      return rc;
    }
  }
  // 4. ghost columns after the receives (transfers receive in place; the loopback study unpacks)
  if (transfer) {
    rc = hdd_comm_wait(comm, stream);
    if (rc) return rc;
    if (side && !offfix && ps != s && comm->kind == hdd_comm::HOST && hipStreamWaitEvent(s, sh->ev_out, 0) != hipSuccess)
      return set_error(HDD_ERR_HIP, "hdd_block_assemble_sharded: wait host transport");
  }
  if (fix_pending) {   // join the off-stream fixup, move its row blocks into place
    e = hipStreamWaitEvent(s, sh->ev_out, 0);
    if (e != hipSuccess) return hip_fail(e, "hdd_block_assemble_sharded: join fixup");
    if (fix_unsupported) return hdd_swipdg_assemble(ctx, &m, kappa, n_comp, tensor, params, pattern, d_vals, stream);
    if (soa)
      return hdd_scatter_fix_q1_soa(ctx, &m, pattern, fbufs.data(), soa_ld, n_comp, sh->d_fix, sh->n_fix, d_vals, stream);
    if (scatter && !soa) return hdd_scatter_fix(ctx, pattern, rb, fbufs.data(), n_comp, sh->d_fix, sh->n_fix, d_vals, stream);
    return HDD_OK;   // in place: the join alone completes the step on `stream`
  }
  if (!transfer) {
    if (ps != s && hipStreamWaitEvent(s, sh->ev_out, 0) != hipSuccess)
      return set_error(HDD_ERR_HIP, "hdd_block_assemble_sharded: wait loopback");
    for (int k = 0; k <= h.n_peers; ++k) h.prefix[k] = sh->recv_prefix[k];
    for (int k = 0; k < h.n_peers; ++k) h.col0[k] = sh->recv_col0[k];
    h.idx = nullptr;
    h.buf = loop_buf;
    e = launch_halo(false, h, s);
    if (e != hipSuccess) return hip_fail(e, "hdd_block_assemble_sharded: unpack");
  }
  // 5. the rows that read a ghost (or everything without overlap)
  if (overlap && split)
    return hdd_swipdg_assemble_tiles(ctx, &m, kappa, n_comp, tensor, params, pattern, d_vals, sh->d_tiles_bd, sh->n_bd,
                                     stream);
  if (overlap) {
    rc = hdd_swipdg_assemble_elements(ctx, &m, kappa, n_comp, tensor, params, pattern, d_vals, sh->d_fix, sh->n_fix,
                                      stream);
    if (rc != HDD_ERR_UNSUPPORTED) return rc;   // (no list kernel for these rules: the whole range again)
  }
  return hdd_swipdg_assemble(ctx, &m, kappa, n_comp, tensor, params, pattern, d_vals, stream);
}

// ------------------------------------------------------------------------------------------------
// watchdog: which stage of the last sharded step has not completed.  A lost peer shows as a step that never
// completes on the device (RCCL waits inside its kernels), so a caller that would block in a device synchronize
// can instead poll these events with a deadline and report the rank and stage before exiting.
// ------------------------------------------------------------------------------------------------
static const char* const stage_names[] = {"complete", "halo pack", "halo exchange (group send/recv)",
                                          "ghost-adjacent element pass", "tile assembly and join"};

extern "C" int hdd_block_step_mark(hdd_shard* sh, void* stream)
{
  if (!sh || sh->host_only) return set_error(HDD_ERR_INVALID, "hdd_block_step_mark: invalid shard");
  hipError_t e = hipSetDevice(sh->device);
  if (e == hipSuccess && !sh->ev_mark) e = hipEventCreateWithFlags(&sh->ev_mark, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventRecord(sh->ev_mark, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "hdd_block_step_mark");
  sh->marked = true;
  return HDD_OK;
}

extern "C" int hdd_block_step_query(hdd_shard* sh, int32_t* stage)
{
  if (!sh || !stage || sh->host_only) return set_error(HDD_ERR_INVALID, "hdd_block_step_query: invalid argument");
  const hipEvent_t evs[4] = {(sh->stages & 1u) ? sh->ev_pack : nullptr, (sh->stages & 2u) ? sh->ev_xdone : nullptr,
                             (sh->stages & 4u) ? sh->ev_out : nullptr, sh->marked ? sh->ev_mark : nullptr};
  *stage = HDD_STAGE_COMPLETE;
  for (int i = 0; i < 4; ++i) {
    if (!evs[i]) continue;
    const hipError_t e = hipEventQuery(evs[i]);
    if (e == hipErrorNotReady) {
      *stage = i + 1;
      return HDD_OK;
    }
    if (e != hipSuccess) return hip_fail(e, "hdd_block_step_query");
  }
  return HDD_OK;
}

extern "C" const char* hdd_block_stage_name(int32_t stage)
{
  return stage >= 0 && stage <= HDD_STAGE_ASSEMBLY ? stage_names[stage] : "unknown stage";
}

extern "C" int hdd_block_step_sync(hdd_shard* sh, void* stream, double timeout_s)
{
  int rc = hdd_block_step_mark(sh, stream);
  if (rc) return rc;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    int32_t st = 0;
    rc = hdd_block_step_query(sh, &st);
    if (rc) return rc;
    if (st == HDD_STAGE_COMPLETE) return HDD_OK;
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (dt > timeout_s) {
      std::string peers;
      for (int32_t p : sh->stage_peers) peers += (peers.empty() ? "" : ", ") + std::to_string(p);
      return set_error(HDD_ERR_TIMEOUT, "rank " + std::to_string(sh->rank) + " of " + std::to_string(sh->nranks) +
                                            ": the sharded step's " + stage_names[st] + " did not complete within " +
                                            std::to_string(timeout_s) + " s (halo peers: " +
                                            (peers.empty() ? "none" : peers) + ")");
    }
    std::this_thread::sleep_for(std::chrono::microseconds(dt < 0.01 ? 20 : 1000));
  }
}
