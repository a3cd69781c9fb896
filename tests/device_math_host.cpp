// Host build of the device math of scenery-insitu_amd/csrc/insitu_device.h (det_log2 / det_exp2 /
// det_pow) for tests/test_device_math.py: prints the bit patterns of the results for the inputs
// given on stdin (one hex word per line), so they can be compared with the oracle's.
#include <cstdio>
#include <cstdint>
#include <cstring>
#include "insitu_device.h"

int main() {
    unsigned a, b;
    char op[8];
    while (std::scanf("%7s %x %x", op, &a, &b) == 3) {
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
