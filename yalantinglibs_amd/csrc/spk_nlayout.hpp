// spk_nlayout.hpp — the op-list interpreter's view of a layout with
// SPK_OP_ARRAY / VARIANT / OPTGROUP / CGROUP / COMPAT / FVAR ops (matching
// ENDs resolved, heap numbering, the first-count screen of a guessed record
// start). Shared by the interpreter kernels (spk_nested.hip) and the tile
// decoder's nested walker (spk_var.hip).
#pragma once
#include "spk_internal.hpp"

namespace spk {

struct NLayout {
  spk_op ops[SPK_MAX_OPS];
  uint8_t heap[SPK_MAX_OPS];  // heap index of a SPAN / OPTION / ARRAY op
  uint8_t end[SPK_MAX_OPS];   // ARRAY: its END; VARIANT: the END of its last alternative
  uint8_t crank[SPK_MAX_OPS]; // COMPAT: its version rank (ops[i].kind is SPK_OP_COMPAT)
  uint32_t n_ops, stride, n_heaps, n_ranks;
  uint32_t fv_cnt, fv_has64, fv_bits;  // USE_FAST_VARINT group: FVAR ops, a 64-bit one, bitset bytes
  // screen of a guessed record start: the first count (SPAN / ARRAY) sits
  // scr_off fixed bytes into the record (~0: no such count before anything
  // data-dependent); its elements take at least scr_esz bytes each
  uint32_t scr_off, scr_esz;
  uint32_t depth;  // deepest nesting of ARRAY / VARIANT / OPTGROUP / CGROUP frames
};

// VARIANT / OPTGROUP / CGROUP: groups placed in the same record, each closed
// by an END (an ARRAY's element ops are one group too, in another record)
__host__ __device__ __forceinline__ bool n_group(uint32_t k) {
  return k == SPK_OP_VARIANT || k == SPK_OP_OPTGROUP || k == SPK_OP_CGROUP;
}

static inline NLayout make_nlayout(const spk_layout *L) {
  NLayout N = {};
  N.n_ops = L->n_ops;
  N.stride = L->rec_stride;
  // open ARRAYs / groups and the groups each one still has to close
  uint32_t stack[SPK_MAX_DEPTH + 1], left[SPK_MAX_DEPTH + 1], d = 0, h = 0;
  for (uint32_t i = 0; i < L->n_ops; ++i) {
    N.ops[i] = L->ops[i];
    const uint32_t k = SPK_OP_KIND(L->ops[i].kind);
    if (k == SPK_OP_COMPAT || k == SPK_OP_CGROUP) {
      N.ops[i].kind = k;
      N.crank[i] = (uint8_t)SPK_OP_RANK(L->ops[i].kind);
      if (N.crank[i] + 1u > N.n_ranks) N.n_ranks = N.crank[i] + 1u;
    }
    if (op_has_heap(k)) N.heap[i] = (uint8_t)h++;
    if (k == SPK_OP_FVAR) {
      ++N.fv_cnt;
      N.fv_has64 |= L->ops[i].size == 8;
    }
    if (k == SPK_OP_ARRAY || n_group(k)) {
      stack[d] = i;
      left[d++] = k == SPK_OP_ARRAY ? 1 : L->ops[i].size;
      if (d > N.depth) N.depth = d;
    }
    if (k == SPK_OP_END && d && --left[d - 1] == 0) N.end[stack[--d]] = (uint8_t)i;
  }
  N.n_heaps = h;
  N.fv_bits = N.fv_cnt ? (N.fv_cnt + 2 + 7) / 8 : 0;
  N.scr_off = ~0u;
  uint32_t pre = 0;
  for (uint32_t i = 0; i < L->n_ops && !N.fv_cnt; ++i) {
    const uint32_t k = SPK_OP_KIND(L->ops[i].kind);
    if (k == SPK_OP_COPY) {
      pre += L->ops[i].size;
      continue;
    }
    if (k == SPK_OP_SPAN || k == SPK_OP_ARRAY) {
      N.scr_off = pre;
      N.scr_esz = k == SPK_OP_SPAN ? L->ops[i].size : 1;
    }
    break;
  }
  return N;
}

}  // namespace spk
