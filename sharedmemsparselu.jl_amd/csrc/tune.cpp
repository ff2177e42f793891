// tune.cpp — the library's environment knobs (struct Tune, plan.hpp; include/smlu.h), read at each
// schedule build / call that uses them (tests change them between handles of one process).
#include <algorithm>
#include <cstdlib>

#include "plan.hpp"

namespace smlu {

Tune tune() {
  Tune v;
  {
    if (const char* e = std::getenv("SMLU_OB")) v.ob = std::max(64, (std::atoi(e) / 64) * 64);
    if (const char* e = std::getenv("SMLU_T128MIN")) v.t128_min = std::atoll(e);
    if (const char* e = std::getenv("SMLU_SMALLK")) v.small_k = std::atoi(e) != 0;
    if (const char* e = std::getenv("SMLU_FULLPIV_NS")) v.fullpiv_ns = std::atoll(e);
    if (const char* e = std::getenv("SMLU_SWEEP_SPIN")) v.sweep_spin = std::atoi(e);
    if (const char* e = std::getenv("SMLU_SOLVE_STEPS")) v.solve_steps = std::atoi(e) == 1;
    v.no_graph = std::getenv("SMLU_NO_GRAPH") != nullptr;
    v.debug_sync = std::getenv("SMLU_DEBUG_SYNC") != nullptr;
    v.no_repivot = std::getenv("SMLU_NO_REPIVOT") != nullptr;
    if (const char* e = std::getenv("OMP_NUM_THREADS")) v.host_threads = std::atoi(e);
  }
  return v;
}

}  // namespace smlu
