// attention_bwd_q.hip — instantiations of the backwardQuery phase (attention_bwd.h).
#include "attention_bwd.h"
#include "mfa_dispatch.h"

namespace mfa {

hipError_t bwd_q_dispatch(const BwdParams& p, int elem, int DP, int ksrc, int vsrc,
                          hipStream_t stream) {
  (void)vsrc;
#define MFA_BQ_CASE(ELEM, DPV, KS)                                                           \
  if (elem == ELEM && DP == DPV && ksrc == KS)                                               \
    return launch_bwd_q<typename ArithOf<ELEM, DPV>::type, DPV, BwdCfg<ELEM, DPV>::BT,       \
                        BwdCfg<ELEM, DPV>::NW, KS>(p, stream);
#define MFA_BQ_DPS(ELEM, KS) \
  MFA_BQ_CASE(ELEM, 32, KS) MFA_BQ_CASE(ELEM, 64, KS) MFA_BQ_CASE(ELEM, 128, KS) MFA_BQ_CASE(ELEM, 256, KS)
  MFA_BQ_DPS(P_FP16, SRC_SAME)
  MFA_BQ_DPS(P_FP16, SRC_I8)
  MFA_BQ_DPS(P_FP16, SRC_I4)
  MFA_BQ_DPS(P_BF16, SRC_SAME)
  MFA_BQ_DPS(P_BF16, SRC_I8)
  MFA_BQ_DPS(P_BF16, SRC_I4)
  MFA_BQ_DPS(P_FP32, SRC_SAME)
#undef MFA_BQ_DPS
#undef MFA_BQ_CASE
  return hipErrorInvalidValue;
}

int bwd_lds_bytes(int kind, int elem, int DP) {
  int bp, bt, nw;
  bwd_block_config(elem, DP, &bp, &bt, &nw);
  const int tile = elem == 0 ? bt * (DP + 1) * 4 : bt * DP * 2;
  return kind == 0 ? 4 * tile : 4 * tile + 4 * bt * 4;
}

}  // namespace mfa
