// mfa_manifest.cpp — the reference's static binding tables, exported through the C ABI.
//
//  * QuantizedKernelLayoutManifest (QuantizedKernelLayoutManifest.swift:8-266): the buffer
//    slot every quantized-attention operand is bound to, per kernel type.  The HIP entry
//    points take the same operands as named arguments; the table is the FFI contract an
//    integrator binding by slot number (the reference's C FFI) keeps using.
//  * The GLUON constants and their enable predicate (AttentionKernel+GluonOptimizations.swift:
//    12-22, :314-320).
#include <cstring>

#include "../../include/mfa/mfa.h"

namespace {

// Slot table (QuantizedKernelLayoutManifest.swift:59-129): data 0-2, output / gradOutput
// share 3, then one slot each in declaration order up to maskBuffer = 30; the scalar metadata
// keys and the scratch buffers have no slot (-1).
int canonical_slot(int key) {
  switch (key) {
    case MFA_QSLOT_Q_DATA: return 0;
    case MFA_QSLOT_K_DATA: return 1;
    case MFA_QSLOT_V_DATA: return 2;
    case MFA_QSLOT_OUTPUT:
    case MFA_QSLOT_GRAD_OUTPUT: return 3;
    case MFA_QSLOT_LOGSUMEXP: return 4;
    case MFA_QSLOT_GRAD_QUERY: return 5;
    case MFA_QSLOT_D_VALUES: return 6;
    case MFA_QSLOT_GRAD_KEY: return 7;
    case MFA_QSLOT_GRAD_VALUE: return 8;
    case MFA_QSLOT_Q_SCALE: return 9;
    case MFA_QSLOT_Q_ZERO_POINT: return 10;
    case MFA_QSLOT_K_SCALE: return 11;
    case MFA_QSLOT_K_ZERO_POINT: return 12;
    case MFA_QSLOT_V_SCALE: return 13;
    case MFA_QSLOT_V_ZERO_POINT: return 14;
    case MFA_QSLOT_DIMS: return 15;
    case MFA_QSLOT_STE_CLIP_RANGE: return 16;
    case MFA_QSLOT_Q_BLOCK_SCALES: return 17;
    case MFA_QSLOT_Q_BLOCK_ZERO_POINTS: return 18;
    case MFA_QSLOT_K_BLOCK_SCALES: return 19;
    case MFA_QSLOT_K_BLOCK_ZERO_POINTS: return 20;
    case MFA_QSLOT_V_BLOCK_SCALES: return 21;
    case MFA_QSLOT_V_BLOCK_ZERO_POINTS: return 22;
    case MFA_QSLOT_Q_PRECOMPUTED_SUMS: return 23;
    case MFA_QSLOT_K_PRECOMPUTED_SUMS: return 24;
    case MFA_QSLOT_V_PRECOMPUTED_SUMS: return 25;
    case MFA_QSLOT_Q_STRIDES: return 26;
    case MFA_QSLOT_K_STRIDES: return 27;
    case MFA_QSLOT_V_STRIDES: return 28;
    case MFA_QSLOT_O_STRIDES: return 29;
    case MFA_QSLOT_MASK_BUFFER: return 30;
    default: return -1;  // maskMetadata (never assigned), numHeads ... scratch1
  }
}

// Which keys each kernel's layout lists (:157-211).  A listed key reports its canonical
// slot (possibly -1 for the metadata keys); an unlisted key reports -1 (Layout.index).
bool listed(int kernel, int key) {
  switch (kernel) {
    case MFA_KERNEL_FORWARD:
      switch (key) {
        case MFA_QSLOT_GRAD_OUTPUT: case MFA_QSLOT_GRAD_QUERY: case MFA_QSLOT_D_VALUES:
        case MFA_QSLOT_GRAD_KEY: case MFA_QSLOT_GRAD_VALUE: case MFA_QSLOT_DIMS:
        case MFA_QSLOT_STE_CLIP_RANGE: case MFA_QSLOT_MASK_METADATA:
          return false;
        default: return true;
      }
    case MFA_KERNEL_BACKWARD_QUERY:
    case MFA_KERNEL_BACKWARD_KEY_VALUE: {
      const bool q = kernel == MFA_KERNEL_BACKWARD_QUERY;
      switch (key) {
        case MFA_QSLOT_Q_DATA: case MFA_QSLOT_K_DATA: case MFA_QSLOT_V_DATA:
        case MFA_QSLOT_GRAD_OUTPUT: case MFA_QSLOT_LOGSUMEXP: case MFA_QSLOT_D_VALUES:
        case MFA_QSLOT_Q_SCALE: case MFA_QSLOT_Q_ZERO_POINT: case MFA_QSLOT_K_SCALE:
        case MFA_QSLOT_K_ZERO_POINT: case MFA_QSLOT_V_SCALE: case MFA_QSLOT_V_ZERO_POINT:
        case MFA_QSLOT_DIMS: case MFA_QSLOT_STE_CLIP_RANGE:
        case MFA_QSLOT_Q_BLOCK_SCALES: case MFA_QSLOT_Q_BLOCK_ZERO_POINTS:
        case MFA_QSLOT_K_BLOCK_SCALES: case MFA_QSLOT_K_BLOCK_ZERO_POINTS:
        case MFA_QSLOT_V_BLOCK_SCALES: case MFA_QSLOT_V_BLOCK_ZERO_POINTS:
        case MFA_QSLOT_Q_STRIDES: case MFA_QSLOT_K_STRIDES: case MFA_QSLOT_V_STRIDES:
        case MFA_QSLOT_O_STRIDES:
          return true;
        case MFA_QSLOT_GRAD_QUERY: return q;
        case MFA_QSLOT_GRAD_KEY: case MFA_QSLOT_GRAD_VALUE: return !q;
        default: return false;
      }
    }
    case MFA_KERNEL_MLA_COMPRESSED:
      switch (key) {
        case MFA_QSLOT_Q_DATA: case MFA_QSLOT_OUTPUT: case MFA_QSLOT_NUM_HEADS:
        case MFA_QSLOT_HEAD_DIMENSION: case MFA_QSLOT_SEQUENCE_LENGTH: case MFA_QSLOT_SCRATCH0:
        case MFA_QSLOT_SCRATCH1:
          return true;
        default: return false;
      }
    default: return false;
  }
}

const char* const kKeyNames[MFA_QSLOT_COUNT] = {
    "qData", "kData", "vData", "output", "gradOutput", "logsumexp", "gradQuery", "dValues",
    "gradKey", "gradValue", "qScale", "qZeroPoint", "kScale", "kZeroPoint", "vScale",
    "vZeroPoint", "dims", "steClipRange", "qBlockScales", "qBlockZeroPoints", "kBlockScales",
    "kBlockZeroPoints", "vBlockScales", "vBlockZeroPoints", "qPrecomputedSums",
    "kPrecomputedSums", "vPrecomputedSums", "qStrides", "kStrides", "vStrides", "oStrides",
    "maskBuffer", "maskMetadata", "numHeads", "numKeyValueHeads", "headDimension",
    "sequenceLength", "scratch0", "scratch1"};

}  // namespace

extern "C" int mfa_quantized_slot(mfa_kernel_type_t kernel, mfa_quantized_slot_key_t key) {
  if ((int)key < 0 || (int)key >= MFA_QSLOT_COUNT || !listed(kernel, key)) return -1;
  return canonical_slot(key);
}

extern "C" int mfa_quantized_slot_table(mfa_kernel_type_t kernel, int32_t* out, int n) {
  if (kernel < MFA_KERNEL_FORWARD || kernel > MFA_KERNEL_MLA_COMPRESSED) return -1;
  int bound = 0;
  for (int k = 0; k < MFA_QSLOT_COUNT; ++k) {
    const int s = mfa_quantized_slot(kernel, (mfa_quantized_slot_key_t)k);
    if (out && k < n) out[k] = s;
    bound += s >= 0;
  }
  return bound;
}

extern "C" const char* mfa_quantized_slot_name(mfa_quantized_slot_key_t key) {
  if ((int)key < 0 || (int)key >= MFA_QSLOT_COUNT) return nullptr;
  return kKeyNames[key];
}

extern "C" void mfa_gluon_constants(uint8_t* split_exp_factor, uint8_t* channel_sync_points,
                                    uint8_t* subtile_size) {
  if (split_exp_factor) *split_exp_factor = MFA_GLUON_SPLIT_EXP_FACTOR;
  if (channel_sync_points) *channel_sync_points = MFA_GLUON_CHANNEL_SYNC_POINTS;
  if (subtile_size) *subtile_size = MFA_GLUON_SUBTILE_SIZE;
}

extern "C" int mfa_gluon_should_enable(uint16_t block_traversal, uint16_t block_head) {
  // shouldEnableGluonOptimizations (:314-320) reads the BLOCK traversal, which every
  // parameter table (the reference's and mfa_dispatch.h's) caps below 512: never true for a
  // plan this library produces, so the standard softmax is the one that runs, as there.
  return block_traversal >= 512 && block_head >= 64;
}
