/*
 * ref_decode_matrix.c -- reaches the reference's own gf_gen_decode_matrix
 * (isa-l_open_src_2.13/erasure_code/erasure_code_base_test.c:133-213, a
 * static function of that test program) for the general-decode parity tests
 * (TEST INFRASTRUCTURE ONLY -- built into oracle/_ref/libisal_ref.so by
 * oracle/Makefile, never linked by the engine).
 *
 * The test program is compiled unmodified where it lies, included into this
 * translation unit so its static function is callable; oracle/Makefile
 * renames its main() on the command line (-Dmain=...) and sizes its matrices
 * for up to 256 rows (-DTEST_SOURCES=256).
 */
#include <stdlib.h>

#include "erasure_code_base_test.c"

/* gf_gen_decode_matrix with src_in_err / nsrcerrs derived from the list, as
 * the test's main() passes them (erasure_code_base_test.c:289-294).
 * Returns 0 or NO_INVERT_MATRIX (-2); decode_index: k entries. */
int ref_gf_gen_decode_matrix(unsigned char *encode_matrix, unsigned char *decode_matrix,
                             unsigned int *decode_index, unsigned char *src_err_list, int nerrs,
                             int k, int m)
{
    unsigned char src_in_err[TEST_SOURCES];
    unsigned char *inv = malloc((size_t)k * k);
    int nsrcerrs = 0, i, rc;
    memset(src_in_err, 0, sizeof src_in_err);
    for (i = 0; i < nerrs; i++) {
        src_in_err[src_err_list[i]] = 1;
        if (src_err_list[i] < k)
            nsrcerrs++;
    }
    rc = gf_gen_decode_matrix(encode_matrix, decode_matrix, inv, decode_index, src_err_list,
                              src_in_err, nerrs, nsrcerrs, k, m);
    free(inv);
    return rc;
}
