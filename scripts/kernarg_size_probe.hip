// Launch latency against the by-value kernel-argument size (measurement tool, not product code): one block writes a
// sequence number to host-mapped memory, the host spins on it; p50 over 3000 launches per size.
// Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/kernarg_size_probe scripts/kernarg_size_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

template <int N>
struct Arg {
    unsigned v[N / 4];
};
template <int N>
__global__ void k_flag(volatile unsigned* host_flag, unsigned seq, Arg<N> b, unsigned* sink) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        sink[0] = b.v[seq % (N / 4)];
        __threadfence_system();
        *host_flag = seq;
    }
}

template <int N>
static double run(hipStream_t s, unsigned* hflag, unsigned* dflag, unsigned* sink, unsigned& seq) {
    Arg<N> a{};
    std::vector<double> t;
    for (int i = 0; i < 3100; ++i) {
        const unsigned q = ++seq;
        a.v[i % (N / 4)] = q;
        const auto t0 = std::chrono::steady_clock::now();
        k_flag<N><<<1, 64, 0, s>>>(dflag, q, a, sink);
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != q) {
        }
        if (i >= 100) t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::nth_element(t.begin(), t.begin() + t.size() / 2, t.end());
    return t[t.size() / 2];
}

int main() {
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    unsigned *hflag, *dflag, *sink;
    (void)hipHostMalloc((void**)&hflag, 64, hipHostMallocMapped | hipHostMallocCoherent);
    (void)hipHostGetDevicePointer((void**)&dflag, hflag, 0);
    (void)hipMalloc(&sink, 64);
    *hflag = 0;
    unsigned seq = 0;
    printf("{");
    printf("\"16\": %.2f, ", run<16>(s, hflag, dflag, sink, seq));
    printf("\"256\": %.2f, ", run<256>(s, hflag, dflag, sink, seq));
    printf("\"512\": %.2f, ", run<512>(s, hflag, dflag, sink, seq));
    printf("\"1024\": %.2f, ", run<1024>(s, hflag, dflag, sink, seq));
    printf("\"1536\": %.2f, ", run<1536>(s, hflag, dflag, sink, seq));
    printf("\"2048\": %.2f, ", run<2048>(s, hflag, dflag, sink, seq));
    printf("\"3072\": %.2f, ", run<3072>(s, hflag, dflag, sink, seq));
    printf("\"4096\": %.2f, ", run<4096>(s, hflag, dflag, sink, seq));
    printf("\"6144\": %.2f, ", run<6144>(s, hflag, dflag, sink, seq));
    printf("\"16_again\": %.2f}\n", run<16>(s, hflag, dflag, sink, seq));
    return 0;
}
