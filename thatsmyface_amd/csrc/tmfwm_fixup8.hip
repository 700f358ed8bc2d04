// dgesdd-route second passes for b = 8 (tmfwm_fixup.h), in a TU of their own so that the
// block sizes compile in parallel.
#include "tmfwm_fixup.h"

namespace tmf {
hipError_t launch_embed_fixup_8(const EmbedArgs &a, const uint32_t *list, const uint32_t *count, int64_t max_entries, hipStream_t st)
{
    return embed_fixup_b<8>(a, list, count, max_entries, st);
}
hipError_t launch_extract_fixup_8(const ExtractArgs &a, const uint32_t *list, const uint32_t *count, int64_t max_entries,
                                   hipStream_t st)
{
    return extract_fixup_b<8>(a, list, count, max_entries, st);
}
}  // namespace tmf
