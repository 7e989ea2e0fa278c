// attention_bwd_kv.hip — instantiations of the backwardKeyValue phase (attention_bwd.h).
#include "attention_bwd.h"
#include "mfa_dispatch.h"

namespace mfa {

hipError_t bwd_kv_dispatch(const BwdParams& p, int elem, int DP, int ksrc, int qsrc,
                           hipStream_t stream) {
  (void)ksrc;
#define MFA_BKV_CASE(ELEM, DPV, QS)                                                          \
  if (elem == ELEM && DP == DPV && qsrc == QS)                                               \
    return launch_bwd_kv<typename ArithOf<ELEM, DPV>::type, DPV, BwdCfg<ELEM, DPV>::BT,      \
                         BwdCfg<ELEM, DPV>::NW, QS>(p, stream);
#define MFA_BKV_DPS(ELEM, QS) \
  MFA_BKV_CASE(ELEM, 32, QS) MFA_BKV_CASE(ELEM, 64, QS) MFA_BKV_CASE(ELEM, 128, QS) MFA_BKV_CASE(ELEM, 256, QS)
  MFA_BKV_DPS(P_FP16, SRC_SAME)
  MFA_BKV_DPS(P_FP16, SRC_I8)
  MFA_BKV_DPS(P_FP16, SRC_I4)
  MFA_BKV_DPS(P_BF16, SRC_SAME)
  MFA_BKV_DPS(P_BF16, SRC_I8)
  MFA_BKV_DPS(P_BF16, SRC_I4)
  MFA_BKV_DPS(P_FP32, SRC_SAME)
#undef MFA_BKV_DPS
#undef MFA_BKV_CASE
  return hipErrorInvalidValue;
}

}  // namespace mfa
