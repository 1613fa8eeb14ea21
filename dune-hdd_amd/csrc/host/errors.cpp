// dune-hdd_amd/csrc/host/errors.cpp -- per-thread last-error message of the C ABI.
#include "hdd.h"
#include "hdd_internal.hh"

namespace hdd {
std::string& last_error_slot()
{
  thread_local std::string msg;
  return msg;
}
int set_error(int code, const std::string& msg)
{
  last_error_slot() = msg;
  return code;
}
}  // namespace hdd

extern "C" int hdd_abi_version(void) { return HDD_ABI_VERSION; }

extern "C" const char* hdd_last_error(const hdd_ctx* /*ctx*/) { return hdd::last_error_slot().c_str(); }

namespace hdd {
const char*& last_tile_kernel_slot()
{
  thread_local const char* name = "";
  return name;
}
}  // namespace hdd

extern "C" const char* hdd_last_tile_kernel(void) { return hdd::last_tile_kernel_slot(); }
