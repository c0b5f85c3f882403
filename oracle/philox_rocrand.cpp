// Test infrastructure: prints Philox4x32-10 outputs computed with rocRAND's own engine
// (/opt/rocm/include/rocrand/rocrand_philox4x32_10.h, host-callable ten_rounds) so the
// oracle's and the kernels' Philox restatement can be pinned against an independent
// implementation.  Usage: philox_rocrand c0 c1 c2 c3 k0 k1   (hex)
#include <rocrand/rocrand_philox4x32_10.h>

#include <cstdio>
#include <cstdlib>

int main(int argc, char** argv) {
    if (argc != 7) return 2;
    unsigned v[6];
    for (int i = 0; i < 6; ++i) v[i] = (unsigned)strtoul(argv[i + 1], nullptr, 16);
    struct Exposed : rocrand_device::philox4x32_10_engine {
        uint4 rounds(uint4 c, uint2 k) { return ten_rounds(c, k); }
    } eng;
    uint4 ctr = {v[0], v[1], v[2], v[3]};
    uint2 key = {v[4], v[5]};
    uint4 o = eng.rounds(ctr, key);
    printf("%08x %08x %08x %08x\n", o.x, o.y, o.z, o.w);
    return 0;
}
