/* oracle.h — TEST ORACLE ONLY.  Prototypes of the plain-C restatement in the
 * oracle C sources.  Symbols carry an ora_ prefix so the oracle can be loaded
 * beside the product library and the reference without clashing. */
#ifndef FQZ5_ORACLE_H
#define FQZ5_ORACLE_H
#include <stdint.h>
#include <stddef.h>

int ora_var_put_u32(uint8_t *cp, const uint8_t *endp, uint32_t v);
int ora_var_get_u32(const uint8_t *cp, const uint8_t *endp, uint32_t *v);

unsigned int ora_rans_compress_bound_4x16(unsigned int size, int order);
uint8_t *ora_rans_compress_to_4x16(uint8_t *in, unsigned int in_size,
                                   uint8_t *out, unsigned int *out_size,
                                   int order);
uint8_t *ora_rans_compress_4x16(uint8_t *in, unsigned int in_size,
                                unsigned int *out_size, int order);
uint8_t *ora_rans_uncompress_to_4x16(uint8_t *in, unsigned int in_size,
                                     uint8_t *out, unsigned int *out_size);
uint8_t *ora_rans_uncompress_4x16(uint8_t *in, unsigned int in_size,
                                  unsigned int *out_size);
/* hts_pack / hts_unpack_meta / hts_unpack (pack.c:56-344), shared */
uint8_t *ora_pack(const uint8_t *d, uint32_t n, uint8_t *meta, int *meta_len, uint32_t *out_len);
int ora_unpack_meta(const uint8_t *d, uint32_t len, uint8_t *map, int *per);
int ora_unpack(const uint8_t *d, uint32_t len, uint8_t *out, uint32_t n, int per,
               const uint8_t *map);

/* arith_dynamic (htscodecs/arith_dynamic.h:41-55) */
unsigned int ora_arith_compress_bound(unsigned int size, int order);
uint8_t *ora_arith_compress_to(uint8_t *in, unsigned int in_size, uint8_t *out,
                               unsigned int *out_size, int order);
uint8_t *ora_arith_uncompress_to(uint8_t *in, unsigned int in_size, uint8_t *out,
                                 unsigned int *out_size);

/* fqzcomp_qual (fork ABI, htscodecs/fqzcomp_qual.h:59-64,155-170) */
typedef struct {
    int num_records;
    uint32_t *len;
    uint32_t *flags;
    unsigned char **seq;
} ora_fqz_slice;

uint8_t *ora_fqz_compress(int vers, ora_fqz_slice *s, uint8_t *in, size_t in_size,
                          size_t *out_size, int strat, void *gp);
uint8_t *ora_fqz_decompress(uint8_t *in, size_t in_size, size_t *out_size,
                            int *lengths, int nlengths, ora_fqz_slice *s);
/* sequence context model, fqzcomp5.c:1073-1406 (encode_seq / decode_seq) */
uint8_t *ora_seq_encode(const uint8_t *in, uint32_t n, const uint32_t *len, int nrec,
                        int both, int k, uint32_t *out_size);
uint8_t *ora_seq_decode(const uint8_t *in, uint32_t in_size, const uint32_t *len, int nrec,
                        int both, int k, uint32_t out_size);
/* LZP pre-pass and the LZP3 sequence method (lzp16e.c, fqzcomp5.c:2013-2021) */
int ora_lzp(const uint8_t *in, int in_len, uint8_t *out);
int ora_unlzp(const uint8_t *in, int in_len, uint8_t *out, int out_cap);
uint8_t *ora_lzp3_compress(uint8_t *in, unsigned int in_size, unsigned int *out_size);
uint8_t *ora_lzp3_uncompress(uint8_t *in, unsigned int in_size, unsigned int u_len,
                             unsigned int *out_size);
#endif
