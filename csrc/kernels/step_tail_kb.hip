// Step-tail instantiations for rows of 5..8 float4 columns (step_tail_kern.h).
#include "step_tail_kern.h"

namespace rocfm {

void launch_tail_group_b(int kp4, const WgradParams& w, const EmbUpdateParams& e, const TailLaunch& l, hipStream_t s) {
  switch (kp4) {
    case 5: launch_tail_kp4<5>(w, e, l, s); break;
    case 6: launch_tail_kp4<6>(w, e, l, s); break;
    case 7: launch_tail_kp4<7>(w, e, l, s); break;
    case 8: launch_tail_kp4<8>(w, e, l, s); break;
    default: throw std::invalid_argument("step_tail: row width outside this unit");
  }
}

}  // namespace rocfm
