// Exhaustive host check of the q8_1 quantizer's division (gguf_q8_1.hpp):
//   fp16(x / d)  ==  fp16(fma(fma(-q, d, x), r, q))  with q = x * r, r within 1 ulp of 1/d
// for every pair of non-negative finite fp16 x, positive finite fp16 d with x <= 256 d
// (|x/d| <= 127.1 inside a q8_1 block, <= 190.5 when d is an fp16 subnormal), and r in
// {rn(1/d), its two neighbours} (v_rcp_f32's 1-ulp bound).  Also d = fp16(amax / 127) against the same form with c = rn(1/127).
// Why it holds: an fp16 quotient is never an fp16 rounding midpoint and stays > 2^-23
// (relative) away from every midpoint, so any fp32 approximation within that distance --
// the corrected quotient is within ~2^-24 -- rounds to the same fp16 value as x/d does.
// Build: g++ -O2 -fopenmp -ffp-contract=off -std=c++17 tools/q81_div_check.cpp -o /tmp/q81_div_check
#include <cmath>
#include <cstdint>
#include <cstdio>

#include "../gguf-triton-kernel_amd/csrc/gguf_half.hpp"

using gq::f2h;
using gq::h2f;

static inline float fast_div(float x, float d, float r)
{
    const float q = x * r;
    const float e = std::fma(-q, d, x);
    return std::fma(e, r, q);
}

int main()
{
    long long bad = 0, pairs = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : bad, pairs)
    for (int db = 1; db < 0x7c00; ++db) {
        const float d = h2f((uint16_t)db);
        const float rn = 1.0f / d;
        const float rs[3] = {rn, std::nextafterf(rn, 0.f), std::nextafterf(rn, INFINITY)};
        for (int xb = 0; xb < 0x7c00; ++xb) {
            const float x = h2f((uint16_t)xb);
            if (x > 256.f * d) break;
            const uint16_t ref = f2h(x / d);
            for (float r : rs) {
                ++pairs;
                if (f2h(fast_div(x, d, r)) != ref) {
                    if (++bad < 10) printf("mismatch x=%a d=%a r=%a\n", x, d, r);
                }
            }
        }
    }
    const float c = 1.0f / 127.0f;
    long long bad_d = 0;
    for (int ab = 1; ab < 0x7c00; ++ab) {
        const float a = h2f((uint16_t)ab);
        if (f2h(fast_div(a, 127.f, c)) != f2h(a / 127.f)) ++bad_d;
    }
    printf("pairs %lld  mismatches %lld  (d = amax/127 mismatches %lld)\n", pairs, bad, bad_d);
    return bad || bad_d;
}
