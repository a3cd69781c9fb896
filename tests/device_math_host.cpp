// Host build of the device math of scenery-insitu_amd/csrc/insitu_device.h (det_log2 / det_exp2 /
// det_pow) for tests/test_device_math.py: prints the bit patterns of the results for the inputs
// given on stdin (one hex word per line), so they can be compared with the oracle's; and the
// closed-form sq_threshold against its defining search over whole ranges of t.
#include <cstdio>
#include <cstdint>
#include <cstring>
#include "insitu_device.h"

// "q lo hi": every float t with bits in [lo, hi] -- sq_threshold (closed form) against
// sq_threshold_search (the definition); prints the number of mismatches
static unsigned check_sq_threshold(uint32_t lo, uint32_t hi) {
    unsigned bad = 0;
    for (uint32_t u = lo;; ++u) {
        float t;
        std::memcpy(&t, &u, 4);
        const float a = insitu::sq_threshold(t), b = insitu::sq_threshold_search(t);
        if (std::memcmp(&a, &b, 4) != 0 && bad++ < 5) std::fprintf(stderr, "sq_threshold mismatch at %08x\n", u);
        if (u == hi) break;
    }
    return bad;
}

int main() {
    unsigned a, b;
    char op[8];
    while (std::scanf("%7s %x %x", op, &a, &b) == 3) {
        if (op[0] == 'q') {
            std::printf("%08x\n", check_sq_threshold(a, b));
            continue;
        }
        float x, y;
        std::memcpy(&x, &a, 4);
        std::memcpy(&y, &b, 4);
        float r = op[0] == 'l' ? insitu::det_log2(x) : (op[0] == 'e' ? insitu::det_exp2(x) : insitu::det_pow(x, y));
        uint32_t u;
        std::memcpy(&u, &r, 4);
        std::printf("%08x\n", u);
    }
    return 0;
}
