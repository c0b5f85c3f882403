// Probe (measurement tool, GPU box): can the host store straight into device memory (large-BAR VRAM)
// so a step's input needs no copy kernel?  Allocates 4 KB of fine-grained / uncached VRAM, reports its
// pointer attributes, writes it from the CPU, and checks a kernel reads the new bytes, for 200 rounds
// (stale-L2 check), timing the host write + kernel round trip.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <immintrin.h>

__global__ void sum_kernel(const volatile float* a, int n, float* out) {
    float s = 0.0f;
    for (int i = threadIdx.x; i < n; i += 64) s += a[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o);
    if (threadIdx.x == 0) *out = s;
}

static int probe(unsigned flags, const char* name) {
    float* d = nullptr;
    if (hipExtMallocWithFlags((void**)&d, 4096, flags) != hipSuccess) {
        printf("%s: alloc failed\n", name);
        return 0;
    }
    hipPointerAttribute_t at{};
    hipError_t e = hipPointerGetAttributes(&at, d);
    printf("%s: dev %p attr rc %d type %d hostPointer %p devicePointer %p\n", name, (void*)d, (int)e, (int)at.type,
           at.hostPointer, at.devicePointer);
    fflush(stdout);
    float* out = nullptr;
    float* hout = nullptr;
    (void)hipHostMalloc((void**)&hout, 64, hipHostMallocMapped | hipHostMallocCoherent);
    (void)hipMalloc((void**)&out, 64);
    float* hp = at.hostPointer ? (float*)at.hostPointer : d;
    int bad = 0;
    double us = 0;
    for (int it = 0; it < 200; ++it) {
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 256; ++i) hp[i] = (float)(it + 1);
        _mm_sfence();
        hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(64), 0, 0, d, 256, out);
        (void)hipMemcpy(hout, out, 4, hipMemcpyDeviceToHost);
        us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        if (hout[0] != 256.0f * (it + 1)) ++bad;
    }
    printf("%s: host-written VRAM read by kernel: %d/200 stale, %.1f us/round\n", name, bad, us / 200);
    fflush(stdout);
    (void)hipFree(d);
    (void)hipFree(out);
    (void)hipHostFree(hout);
    return 1;
}

int main() {
    probe(hipDeviceMallocFinegrained, "finegrained");
    probe(hipDeviceMallocUncached, "uncached");
    return 0;
}
