// quant_device.hip -- GGUF weight quantizers on the device (on-device
// requantization).  Each thread produces one block with the host producers' exact code
// (quant/gguf_quant_blocks.hpp: the reference's float operation order, contraction off, IEEE
// divide/sqrt), so the bytes equal gq_quantize_* on the host and the reference's
// utils/quantize producers.  The K-quant search is scalar and data-dependent (21 / 19 candidate
// scales per sub-block): a thread per super-block, 64-thread workgroups, its arrays in scratch.
#include <hip/hip_runtime.h>

#include "gguf_internal.hpp"
#include "quant/gguf_quant_blocks.hpp"

namespace gq {
namespace {

// F: 0 = Q8_0 (fp16 in, 34 B), 1 = Q4_K (fp32 in, 144 B), 2 = Q6_K (fp32 in, 210 B), 3 = Q8_1 (fp16 in, 36 B)
template <int F>
__global__ __launch_bounds__(64) void quant_blocks_kernel(const void *__restrict__ x, uint8_t *__restrict__ y, int64_t nblocks)
{
    const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (b >= nblocks) return;
    if constexpr (F == 0) qblk::q8_block<false>((const uint16_t *)x + b * 32, y + b * 34);
    else if constexpr (F == 1) qblk::q4k_block((const float *)x + b * 256, y + b * 144);
    else if constexpr (F == 2) qblk::q6k_block((const float *)x + b * 256, y + b * 210);
    else qblk::q8_block<true>((const uint16_t *)x + b * 32, y + b * 36);
}

} // namespace

hipError_t launch_quant_blocks(int kind, const void *x, void *y, int64_t nblocks, hipStream_t s)
{
    if (nblocks <= 0) return hipSuccess;
    const dim3 grid((unsigned)((nblocks + 63) / 64)), block(64);
    switch (kind) {
    case 0: quant_blocks_kernel<0><<<grid, block, 0, s>>>(x, (uint8_t *)y, nblocks); break;
    case 1: quant_blocks_kernel<1><<<grid, block, 0, s>>>(x, (uint8_t *)y, nblocks); break;
    case 2: quant_blocks_kernel<2><<<grid, block, 0, s>>>(x, (uint8_t *)y, nblocks); break;
    case 3: quant_blocks_kernel<3><<<grid, block, 0, s>>>(x, (uint8_t *)y, nblocks); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

} // namespace gq
