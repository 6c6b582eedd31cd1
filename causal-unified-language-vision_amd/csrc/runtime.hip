// C-ABI plumbing shared by every kernel file: thread-local last-error string and the launch
// check. Nothing here allocates device memory or synchronises (SURVEY.md §8(b) "Ownership").
#include "common.h"

static thread_local std::string g_last_error;

void cullavo_set_error(const std::string& msg) { g_last_error = msg; }

int cullavo_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return CULLAVO_EHIP;
  }
  return CULLAVO_OK;
}

extern "C" int cullavo_abi_version(void) { return CULLAVO_ABI_VERSION; }
extern "C" const char* cullavo_last_error(void) { return g_last_error.c_str(); }
