#include "dsort_internal.h"
namespace dsort {
int set_err(dsort_ctx *, int code, const std::string &) { return code; }
int hip_err(dsort_ctx *, hipError_t, const char *) { return -3; }
int ensure(dsort_ctx *, void **, size_t *, size_t, const char *) { return -2; }
}
namespace dsort {
void fault_point(hipStream_t, int) {}
}
