// Host-visible output latency against the way a kernel writes N 8-byte words to host-mapped memory (measurement tool,
// not product code): one block of 256 threads, lane i stores word i; the host spins until it sees all of them (tagged
// forms: every word carries the sequence number in its high half) or the flag.  p50 over 3000 launches, in us.
//   tag8    8-byte system-scope relaxed atomic stores of tagged words (the step outputs' form)
//   tag16   the same words stored in pairs, 16-byte system-coherent (sc0 sc1) vector stores (lanes 0..N/2)
//   plain   plain 8-byte stores, every wave's vmcnt(0), barrier, __threadfence_system, then a flag word
// Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/hostwrite_probe scripts/hostwrite_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

enum { TAG8, TAG16, PLAIN };

template <int MODE>
__global__ void __launch_bounds__(256) k_out(uint64_t* out, unsigned* flag, unsigned seq, int n) {
    const int i = threadIdx.x;
    if (MODE == TAG8) {
        for (int w = i; w < n; w += 256)
            __hip_atomic_store(out + w, ((uint64_t)seq << 32) | (uint32_t)w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (MODE == TAG16) {
        for (int w = 2 * i; w < n; w += 512) {
            const uint64_t a = ((uint64_t)seq << 32) | (uint32_t)w, b = ((uint64_t)seq << 32) | (uint32_t)(w + 1);
            __attribute__((ext_vector_type(4))) unsigned v = {(unsigned)a, (unsigned)(a >> 32), (unsigned)b,
                                                              (unsigned)(b >> 32)};
            // a 16-byte vector store, system-coherent write-through (sc0 sc1), as the 8-byte atomic stores above
            asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(out + w), "v"(v) : "memory");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        for (int w = i; w < n; w += 256) out[w] = ((uint64_t)seq << 32) | (uint32_t)w;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (i == 0) {
            __threadfence_system();
            __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

template <int MODE>
static double run(hipStream_t s, uint64_t* h, uint64_t* d, unsigned* hf, unsigned* df, int n, unsigned& seq) {
    std::vector<double> t;
    for (int it = 0; it < 3100; ++it) {
        const unsigned q = ++seq;
        const auto t0 = std::chrono::steady_clock::now();
        k_out<MODE><<<1, 256, 0, s>>>(d, df, q, n);
        bool ok = true;  // bounded spins: a form whose words never reach the host reports -1
        if (MODE == PLAIN) {
            while (ok && __atomic_load_n(hf, __ATOMIC_ACQUIRE) != q)
                ok = std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(200);
        } else {
            for (int w = n - 1; ok && w >= 0; --w)
                while (ok && (uint32_t)(__atomic_load_n(h + w, __ATOMIC_ACQUIRE) >> 32) != q)
                    ok = std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(200);
        }
        if (!ok) {
            (void)hipStreamSynchronize(s);
            return -1.0;
        }
        if (it >= 100) t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    (void)hipStreamSynchronize(s);
    std::nth_element(t.begin(), t.begin() + t.size() / 2, t.end());
    return t[t.size() / 2];
}

int main() {
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    uint64_t *h, *d;
    unsigned *hf, *df;
    (void)hipHostMalloc((void**)&h, 8 * 2048, hipHostMallocMapped | hipHostMallocCoherent);
    (void)hipHostGetDevicePointer((void**)&d, h, 0);
    (void)hipHostMalloc((void**)&hf, 64, hipHostMallocMapped | hipHostMallocCoherent);
    (void)hipHostGetDevicePointer((void**)&df, hf, 0);
    unsigned seq = 0;
    printf("{");
    const int ns[] = {2, 64, 184, 512, 1456};
    for (int k = 0; k < 5; ++k) {
        const int n = ns[k];
        const double a = run<TAG8>(s, h, d, hf, df, n, seq);
        const double b = run<TAG16>(s, h, d, hf, df, n, seq);
        const double c = run<PLAIN>(s, h, d, hf, df, n, seq);
        printf("%s\"n%d\": {\"tag8\": %.2f, \"tag16\": %.2f, \"plain_fence_flag\": %.2f}", k ? ", " : "", n, a, b, c);
    }
    printf("}\n");
    return 0;
}
