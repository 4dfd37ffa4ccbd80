// stage3_cpu_lib.cpp -- TEST / BASELINE INFRASTRUCTURE ONLY (oracle/_build/libstage3_cpu.so).
// The error channel of the CPU build of the stage-3 pass (the product sets it
// through gsnapdp__set_err, gsnapdp_kernels.hip).
#include <string>

static thread_local std::string g_err;
void gsnapdp__set_err(const std::string& s) { g_err = s; }
extern "C" const char* s3cpu_last_error(void) { return g_err.c_str(); }
