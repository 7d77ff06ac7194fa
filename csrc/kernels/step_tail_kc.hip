// Step-tail instantiations for rows of 9..12 float4 columns (step_tail_kern.h).
#include "step_tail_kern.h"

namespace rocfm {

void launch_tail_group_c(int kp4, const WgradParams& w, const EmbUpdateParams& e, const TailLaunch& l, hipStream_t s) {
  switch (kp4) {
    case 9: launch_tail_kp4<9>(w, e, l, s); break;
    case 10: launch_tail_kp4<10>(w, e, l, s); break;
    case 11: launch_tail_kp4<11>(w, e, l, s); break;
    case 12: launch_tail_kp4<12>(w, e, l, s); break;
    default: throw std::invalid_argument("step_tail: row width outside this unit");
  }
}

}  // namespace rocfm
