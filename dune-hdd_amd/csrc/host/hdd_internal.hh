// dune-hdd_amd/csrc/host/hdd_internal.hh -- error plumbing shared by the host and device halves of the ABI.
// The reference reports failures with DUNE_THROW (swipdg.hh:173-176, base.hh:285-289); across the C ABI
// they become status codes plus a per-thread message (hdd_last_error).
#pragma once
#include <string>

#include "hdd.h"

namespace hdd {
std::string& last_error_slot();
// name of the assembly kernel the last hdd_swipdg_assemble call on this thread launched (hdd_last_tile_kernel; every
// launch path sets it, element-list side passes keep the tile launch's): static strings only
const char*& last_tile_kernel_slot();
int set_error(int code, const std::string& msg);
int ctx_device(const hdd_ctx* ctx);   // HIP device ordinal a context is bound to
}  // namespace hdd

// Sharded-step fixup off the assembly stream (abi_device.hip, used by shard.hip): the element-list pass into side
// buffers of hdd_fix_rb(elem_type) doubles per listed element (n + 1 slots per component), and the copy of those
// row blocks into the value arrays.
int hdd_fix_rb(int32_t elem_type);
int hdd_assemble_elements_buf(hdd_ctx* ctx, const hdd_mesh* m, const hdd_scalar_fn* kappa, int32_t n_comp,
                              const hdd_tensor_fn* tensor, const hdd_swipdg_params* p, const hdd_csr* pattern,
                              double* const* d_bufs, const int32_t* d_elems, int64_t n_elems, void* stream);
int hdd_scatter_fix(hdd_ctx* ctx, const hdd_csr* pattern, int32_t rb, double* const* d_bufs, int32_t n_comp,
                    const int32_t* d_elems, int64_t n_elems, double* const* d_vals, void* stream);
// Q1 side buffers in value-major (SoA) order: value k (canonical: row i, block b, column c, k = 20 i + 4 b + c) of
// listed element j at d_bufs[c][k ld + j] (coalesced element-pass stores), put into place by a wave per element;
// and a full-range launch that leaves reserve_wg workgroup slots to that element pass
int hdd_assemble_elements_soa(hdd_ctx* ctx, const hdd_mesh* m, const hdd_scalar_fn* kappa, int32_t n_comp,
                              const hdd_tensor_fn* tensor, const hdd_swipdg_params* p, const hdd_csr* pattern,
                              double* const* d_bufs, int64_t ld, const int32_t* d_elems, int64_t n_elems, void* stream);
int hdd_scatter_fix_q1_soa(hdd_ctx* ctx, const hdd_mesh* m, const hdd_csr* pattern, double* const* d_bufs, int64_t ld,
                           int32_t n_comp, const int32_t* d_elems, int64_t n_elems, double* const* d_vals, void* stream);
int hdd_assemble_reserve(hdd_ctx* ctx, const hdd_mesh* m, const hdd_scalar_fn* kappa, int32_t n_comp,
                         const hdd_tensor_fn* tensor, const hdd_swipdg_params* p, const hdd_csr* pattern,
                         double* const* d_vals, void* stream, int32_t reserve_wg);
// the same pass in place (no side buffer), beside a full-range assembly that skips those elements' row blocks
int hdd_assemble_elements_inplace(hdd_ctx* ctx, const hdd_mesh* m, const hdd_scalar_fn* kappa, int32_t n_comp,
                                  const hdd_tensor_fn* tensor, const hdd_swipdg_params* p, const hdd_csr* pattern,
                                  double* const* d_vals, const int32_t* d_elems, int64_t n_elems, void* stream);
// reserve_wg: workgroups of the concurrent element pass (in-place fixup) -- the persistent launch leaves that many
// slots free when its own tiles would fill the CUs (launch_persistent)
int hdd_assemble_skip_ghost(hdd_ctx* ctx, const hdd_mesh* m, const hdd_scalar_fn* kappa, int32_t n_comp,
                            const hdd_tensor_fn* tensor, const hdd_swipdg_params* p, const hdd_csr* pattern,
                            double* const* d_vals, void* stream, int32_t reserve_wg = 0);
