// Largest by-value kernel argument this HIP runtime accepts (measurement tool, not product code).
// Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/kernarg_probe scripts/kernarg_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
template <int NB>
struct Blob {
    unsigned char b[NB];
};
template <int NB>
__global__ void k(const Blob<NB> a, int* out) {
    if (threadIdx.x == 0) out[0] = a.b[NB - 1] + a.b[0];
}
template <int NB>
void run(int* d) {
    Blob<NB> a{};
    a.b[0] = 1;
    a.b[NB - 1] = 2;
    hipLaunchKernelGGL(k<NB>, dim3(1), dim3(64), 0, 0, a, d);
    hipError_t e = hipDeviceSynchronize();
    int h = -1;
    if (e == hipSuccess) e = hipMemcpy(&h, d, sizeof(int), hipMemcpyDeviceToHost);
    printf("{\"bytes\": %d, \"err\": \"%s\", \"value\": %d}\n", NB, hipGetErrorString(e), h);
    (void)hipGetLastError();
}
int main() {
    int* d;
    if (hipMalloc(&d, sizeof(int)) != hipSuccess) return 1;
    run<3072>(d);
    run<4000>(d);
    run<4096>(d);
    run<4600>(d);
    run<6000>(d);
    run<8192>(d);
    return 0;
}
