// Exit probe (tools/diag/exit_probe.sh): the smallest hipcc-built shared library with one kernel, loaded by Python
// with ctypes, to tell a rocprofv3 exit-time fault of ANY such library from one of libgol_hip.so.
#include <hip/hip_runtime.h>

__global__ void tiny_kernel(int* p) { p[threadIdx.x] = threadIdx.x; }

extern "C" int tiny_run() {
    int* d = nullptr;
    if (hipMalloc(&d, 64 * sizeof(int)) != hipSuccess) return 1;
    tiny_kernel<<<1, 64>>>(d);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    return hipFree(d) == hipSuccess ? 0 : 3;
}
