/* pkt_oracle.h — CPU oracle (TEST INFRASTRUCTURE ONLY; see pkt_oracle.c header).
 * Uses the schema of include/pktgpu.h (pkt_batch_t / pkt_out_t with HOST pointers). */
#ifndef PKT_ORACLE_H
#define PKT_ORACLE_H
#include "../include/pktgpu.h"

#ifdef __cplusplus
extern "C" {
#endif
const char *orc_hdr_name(int t);
int orc_hdr_size(int t);
int orc_hdr_field_count(int t);
int orc_hdr_field(int t, int i, const char **name, uint16_t *start, uint16_t *end);
uint64_t orc_bit_range(const uint8_t *map, size_t msb, size_t lsb);
void orc_bytes(const uint8_t *map, size_t msb, size_t lsb, uint8_t *out);
uint16_t orc_ipv4_checksum(const uint8_t *v, size_t len);
int orc_parse_one(const uint8_t *p, size_t len, int entry, const pkt_out_t *out, uint64_t i, uint64_t n);
int orc_parse_batch(const pkt_batch_t *b, int entry, const pkt_out_t *out, int nthreads);
int orc_extract_fields(const pkt_batch_t *b, const pkt_chain_t *chain, const pkt_field_spec_t *specs,
                       uint32_t nspec, uint64_t *const *values, uint8_t *const *found);
void orc_set_bit_range(uint8_t *map, size_t msb, size_t lsb, uint64_t value);
int orc_set_fields(const pkt_batch_t *b, const pkt_chain_t *chain, const pkt_field_spec_t *specs,
                   uint32_t nspec, const uint64_t *const *values);
int orc_ipv4_update_checksum(const pkt_batch_t *b, const pkt_chain_t *chain, uint32_t occurrence);
int orc_pktgen_loop(const uint8_t *tpl, size_t len, int entry, int mode, uint64_t first, uint64_t cnt,
                    uint8_t *out, size_t stride, int nthreads);
long orc_slow_parse_to_vec(const uint8_t *p, size_t len, int entry, uint8_t *out, size_t cap);
int orc_round_trip_batch(const pkt_batch_t *b, int entry, int slow, uint8_t *dst, uint64_t dst_len,
                         uint32_t *out_len, int nthreads);
#ifdef __cplusplus
}
#endif
#endif
