// dune-hdd_amd/csrc/host/hdd_internal.hh -- error plumbing shared by the host and device halves of the ABI.
// The reference reports failures with DUNE_THROW (swipdg.hh:173-176, base.hh:285-289); across the C ABI
// they become status codes plus a per-thread message (hdd_last_error).
#pragma once
#include <string>

#include "hdd.h"

namespace hdd {
std::string& last_error_slot();
int set_error(int code, const std::string& msg);
int ctx_device(const hdd_ctx* ctx);   // HIP device ordinal a context is bound to
}  // namespace hdd
