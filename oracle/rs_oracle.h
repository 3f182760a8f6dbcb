/* rs_oracle.h -- CPU restatement of the ISA-L 2.13 RS path (TEST INFRASTRUCTURE ONLY). */
#ifndef RS_ORACLE_H
#define RS_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
void orc_init(void);
uint8_t orc_gf_mul(uint8_t a, uint8_t b);
uint8_t orc_gf_inv(uint8_t a);
uint8_t orc_gf_exp(int i);
void orc_gen_rs_matrix(uint8_t *a, int m, int k);
void orc_gen_cauchy1_matrix(uint8_t *a, int m, int k);
int orc_invert_matrix(uint8_t *in, uint8_t *out, int n);
void orc_vect_mul_init(uint8_t c, uint8_t *tbl);
void orc_init_tables(int k, int rows, const uint8_t *a, uint8_t *gftbls);
void orc_encode_data(int len, int srcs, int dests, const uint8_t *v,
                     uint8_t *const *src, uint8_t *const *dest);
void orc_encode_data_update(int len, int k, int rows, int vec_i, const uint8_t *v,
                            const uint8_t *data, uint8_t *const *dest);
void orc_vect_mul(int len, const uint8_t *a, const uint8_t *src, uint8_t *dest);
void orc_encode_block(int k, int e, int len, uint8_t *const *data, uint8_t *const *parity);
int orc_decode_block(int k, int e, int len, const uint8_t *err_list,
                     uint8_t *const *data, uint8_t *const *parity, uint8_t *const *out);
int orc_decode_matrix(int k, int e, const uint8_t *err_list, uint8_t *c_out);
int orc_gen_decode_matrix(const uint8_t *encode_matrix, int k, int m, const uint8_t *err_list,
                          int nerrs, uint8_t *decode_matrix, int *decode_index);
int orc_decode_general(const uint8_t *encode_matrix, int k, int m, int len,
                       const uint8_t *err_list, int nerrs, uint8_t *const *rows,
                       uint8_t *const *out);
uint64_t orc_synth_word(uint64_t seed, uint64_t row, uint64_t word);
void orc_synth_row(uint64_t seed, uint64_t row, uint8_t *dst, size_t len);
void orc_erasure_pattern(uint64_t seed, uint64_t blk, int k, int e, uint8_t *err_list);
#ifdef __cplusplus
}
#endif
#endif
