// ABI housekeeping: version and per-thread error text.
#include <cstdarg>
#include <cstdio>

#include "vm_common.h"

namespace vm {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace vm

extern "C" int vm_abi_version(void) { return VM_ABI_VERSION; }
extern "C" const char* vm_last_error(void) { return vm::g_err; }
