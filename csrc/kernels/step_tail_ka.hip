// Step-tail instantiations for rows of 1..4 float4 columns (step_tail_kern.h).
#include "step_tail_kern.h"

namespace rocfm {

void launch_tail_group_a(int kp4, const WgradParams& w, const EmbUpdateParams& e, const TailLaunch& l, hipStream_t s) {
  switch (kp4) {
    case 1: launch_tail_kp4<1>(w, e, l, s); break;
    case 2: launch_tail_kp4<2>(w, e, l, s); break;
    case 3: launch_tail_kp4<3>(w, e, l, s); break;
    case 4: launch_tail_kp4<4>(w, e, l, s); break;
    default: throw std::invalid_argument("step_tail: row width outside this unit");
  }
}

}  // namespace rocfm
