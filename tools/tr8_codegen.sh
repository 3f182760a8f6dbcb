# Instruction mix of bitslice.h tr8 as hipcc emits it for gfx950 (tool, not
# product): one load -> tr8 -> store kernel, device assembly only.
#   bash tools/tr8_codegen.sh   -> 24 v_bitop3_b32, 6 v_lshrrev_b64, 6 v_lshlrev_b64
set -e
D=$(mktemp -d)
cat > $D/t.hip <<'K'
#include "bitslice.h"
using namespace rsgpu::bs;
__global__ void k_tr8(const uint8_t* in, uint8_t* out)
{
    uint32_t W[8];
    const long long off = (blockIdx.x * 64 + threadIdx.x) * 32;
    load32(in, off, true, W);
    tr8(W, vconst(0x0F0F0F0Fu), vconst(0x33333333u), vconst(0x55555555u));
    store32(out, off, W);
}
K
/opt/rocm/bin/hipcc -O3 -std=c++20 --offload-arch=gfx950 -I$(dirname $0)/../storage-benchmarks_amd/csrc \
    --cuda-device-only -S $D/t.hip -o $D/t.s 2>/dev/null
awk '/^_Z5k_tr8/,/s_endpgm/' $D/t.s | grep -E "^\s+v_" | awk '{print $1}' | sort | uniq -c
rm -rf $D
