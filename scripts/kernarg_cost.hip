// Host-side cost of launching a kernel with a by-value argument of S bytes (measurement tool, not product code):
// per size, the mean wall time of the launch call alone (2000 back-to-back launches of a one-wave kernel) and of a
// launch + completion round trip (the kernel stores a sequence word into host-mapped memory, the host spins).
// Build: hipcc --offload-arch=gfx950 -O2 -o scripts/kernarg_cost scripts/kernarg_cost.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
template <int NB>
struct Blob {
    unsigned char b[NB];
};
template <int NB>
__global__ void k(const Blob<NB> a, unsigned* flag, unsigned seq) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq + a.b[NB - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <int NB>
void run(unsigned* flag, hipStream_t s) {
    Blob<NB> a{};
    for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k<NB>, dim3(1), dim3(64), 0, s, a, flag, 0u);
    (void)hipStreamSynchronize(s);
    const int n = 2000;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k<NB>, dim3(1), dim3(64), 0, s, a, flag, 0u);
    auto t1 = std::chrono::steady_clock::now();
    (void)hipStreamSynchronize(s);
    double rt = 0;
    for (unsigned i = 1; i <= (unsigned)n; ++i) {
        auto r0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(k<NB>, dim3(1), dim3(64), 0, s, a, flag, 1000000u + i);
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != 1000000u + i) {
        }
        rt += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - r0).count();
    }
    (void)hipStreamSynchronize(s);
    printf("{\"arg_bytes\": %d, \"launch_call_us\": %.3f, \"round_trip_us\": %.3f}\n", NB,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / n, rt / n);
}
int main() {
    unsigned* flag;
    if (hipHostMalloc((void**)&flag, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
    *flag = 0;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
    run<16>(flag, s);
    run<256>(flag, s);
    run<1536>(flag, s);
    run<2048>(flag, s);
    run<3328>(flag, s);
    run<4096>(flag, s);
    return 0;
}
