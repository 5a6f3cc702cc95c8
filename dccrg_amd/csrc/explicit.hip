// explicit.hip -- grids with mixed refinement levels (placeholder until the
// device hash + CSR neighbor build lands).
#include "grid.hpp"

namespace dccrgx {

int explicit_create(dccrgx_grid*, const uint64_t*, size_t)
{
    return set_error(DCCRGX_EINVAL, "mixed-level grids are not supported yet");
}
void explicit_destroy(dccrgx_grid*) {}
int explicit_build_hood(dccrgx_grid*, Hood&) { return set_error(DCCRGX_EINVAL, "unsupported"); }
int explicit_get_cells(const dccrgx_grid*, const Hood&, int32_t, uint64_t*, size_t, size_t*)
{
    return set_error(DCCRGX_EINVAL, "unsupported");
}
int explicit_slots_of(const dccrgx_grid*, const uint64_t*, size_t, int64_t*, hipStream_t)
{
    return set_error(DCCRGX_EINVAL, "unsupported");
}
int explicit_neighbors_of(const dccrgx_grid*, const Hood&, const uint64_t*, size_t, uint64_t*, uint64_t*,
                          int32_t*, size_t, hipStream_t)
{
    return set_error(DCCRGX_EINVAL, "unsupported");
}
int explicit_neighbors_to(const dccrgx_grid*, const Hood&, const uint64_t*, size_t, uint64_t*, uint64_t*,
                          size_t, hipStream_t)
{
    return set_error(DCCRGX_EINVAL, "unsupported");
}
int explicit_gol(dccrgx_grid*, const Hood&, const Field&, const Field&, const Field&, int32_t, hipStream_t)
{
    return set_error(DCCRGX_EINVAL, "unsupported");
}

}  // namespace dccrgx
