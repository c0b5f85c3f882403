// Test infrastructure: prints Threefry-2x32-20 outputs computed with rocRAND's own engine
// (/opt/rocm/include/rocrand/rocrand_threefry2x32_20.h, host-callable threefry_rounds), so the oracle's
// and the kernels' Threefry restatement (oracle/jax_random_oracle.py, csrc/srbd_jaxrng.h) can be pinned
// against an independent implementation.  Reads lines "x0 x1 k0 k1" (hex) on stdin, writes "y0 y1".
#include <rocrand/rocrand_threefry2x32_20.h>

#include <cstdio>

int main() {
    struct Exposed : rocrand_device::threefry2x32_20_engine {
        static uint2 rounds(uint2 c, uint2 k) { return threefry_rounds(c, k); }
    };
    unsigned v[4];
    while (scanf("%x %x %x %x", &v[0], &v[1], &v[2], &v[3]) == 4) {
        const uint2 o = Exposed::rounds(uint2{v[0], v[1]}, uint2{v[2], v[3]});
        printf("%08x %08x\n", o.x, o.y);
    }
    return 0;
}
