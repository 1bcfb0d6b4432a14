// m3_inst.hip -- one board configuration's kernels + launchers (m3_kernels.hpp),
// compiled once per configuration: -DM3_INST=<id> (0 .. N_CONFIGS - 1).
#include "m3_kernels.hpp"

#ifndef M3_INST
#error "compile with -DM3_INST=<configuration id>"
#endif
#define M3_CAT_(a, b) a##b
#define M3_CAT(a, b) M3_CAT_(a, b)

namespace m3k {
M3_INSTANTIATE(template, M3_CAT(CF_, M3_INST))
}  // namespace m3k

#ifdef M3_PHASE_PROF
extern "C" int M3_CAT(m3_prof_read_, M3_INST)(uint64_t* out, int reset) { return m3_prof_read_tu(out, reset); }
#endif
