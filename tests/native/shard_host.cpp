// Host build of the list passes' segment layout (tmfwm_internal.h shard_base) for
// tests/test_list_segments.py: segment s must hold exactly the block rows r < rows with
// r % kListShards == s, nbw slots per row, the segments back to back from 0 to rows * nbw.
#include "../../thatsmyface_amd/csrc/tmfwm_internal.h"

extern "C" int shard_check(uint32_t rows, uint32_t nbw)
{
    using namespace tmf;
    if (shard_base(0, rows, nbw) != 0) return 1;
    if (shard_base(kListShards, rows, nbw) != rows * nbw) return 2;
    for (uint32_t s = 0; s < kListShards; ++s) {
        const uint32_t rows_s = s < rows ? (rows - 1 - s) / kListShards + 1 : 0;
        if (shard_base(s + 1, rows, nbw) - shard_base(s, rows, nbw) != rows_s * nbw) return 3;
    }
    return 0;
}

extern "C" uint32_t shard_count() { return tmf::kListShards; }
