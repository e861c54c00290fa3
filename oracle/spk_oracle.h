/*
 * spk_oracle.h — CPU restatement of struct_pack's wire format for the
 * record model of include/spk_codec.h.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * of the HIP codec — never as the thing measured or shipped. The product
 * library (yalantinglibs_amd/libspk_codec.so) does not link it.
 *
 * Parity of this restatement is pinned against the reference itself:
 * tests/golden/ holds byte fixtures and digests produced by
 * oracle/_ref/golden_gen, a program compiled from the unmodified reference
 * headers (tests/test_oracle_golden.py).
 */
#ifndef SPK_ORACLE_H
#define SPK_ORACLE_H
#include "../include/spk_codec.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Host pointers throughout. Return SPK_OK / SPK_E_*. */
int spko_plan(const spk_layout *L, int mode, uint64_t n, const void *recs,
              const void *const *heaps, spk_plan_t *plan);
int spko_encode(const spk_layout *L, int mode, uint64_t n, const void *recs,
                const void *const *heaps, void *out, uint64_t out_cap,
                uint64_t *msg_offsets, uint64_t *written);
/* body bytes of records [0,n) at an imposed width (no header/count):
 * the per-shard piece of a multi-GPU single message. */
int spko_encode_body(const spk_layout *L, uint64_t n, const void *recs,
                     const void *const *heaps, unsigned width, void *out,
                     uint64_t out_cap, uint64_t *written);
int spko_decode(const spk_layout *L, int mode, const void *wire,
                uint64_t wire_len, const uint64_t *msg_offsets, uint64_t n_msgs,
                void *recs, uint64_t rec_cap, void *const *heaps,
                const uint64_t *heap_caps, spk_dresult_t *res, int32_t *errc);

#ifdef __cplusplus
}
#endif
#endif
