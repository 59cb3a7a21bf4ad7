/* ORACLE — TEST INFRASTRUCTURE ONLY (see keccak_ref.c header). */
#ifndef PRYSM_AMD_ORACLE_H
#define PRYSM_AMD_ORACLE_H
#include <stdint.h>

void or_keccak_f1600(uint64_t A[25]);
void or_keccak_f1600_unrolled(uint64_t A[25]);
int or_set_fast_permutation(int on);
void or_sponge(const uint8_t* in, uint64_t len, uint8_t pad, uint32_t rate, uint8_t* out,
               uint32_t out_len);
void or_keccak256(const uint8_t* in, uint64_t len, uint8_t out[32]);
void or_sha3_256(const uint8_t* in, uint64_t len, uint8_t out[32]);
void or_keccak256_batch(const uint8_t* in, uint64_t n, uint32_t msg_len, uint8_t* out, int nthreads);
void or_keccak256_var(const uint8_t* in, const uint64_t* offs, uint64_t n, uint8_t* out);

uint64_t or_splitmix64_word(uint64_t seed, uint64_t k);
void or_fill_splitmix(uint8_t* out, uint64_t nbytes, uint64_t seed, uint64_t word0);

int or_merkle_hash(const uint8_t* items, uint64_t n, uint32_t item_len, uint8_t out[32], int nthreads);
int or_merkle_hash_var(const uint8_t* data, const uint64_t* offs, uint64_t n, uint8_t out[32]);
int or_merkle_hash_gen(uint64_t n, uint32_t item_len, uint64_t seed, uint8_t out[32], int nthreads);
int or_merkle_nodes(const uint8_t* nodes, uint64_t count, uint64_t n_total, uint8_t out[32], int nthreads);
int or_merkle_subtree_gen(uint64_t n, uint32_t item_len, uint64_t seed, uint64_t shard,
                          uint32_t shard_height, uint8_t out[32], int nthreads);

int or_deposit_trie_build(const uint8_t* data, const uint64_t* offs, uint64_t n, uint32_t depth,
                          uint8_t* levels_out, uint8_t root[32]);
int or_deposit_trie_incremental(const uint8_t* data, const uint64_t* offs, uint64_t n, uint32_t depth,
                                uint8_t root[32]);
int or_verify_merkle_branch(const uint8_t leaf[32], const uint8_t* branch, uint32_t depth,
                            uint64_t index, uint32_t tree_depth, const uint8_t root[32]);
int or_merkle_root(const uint8_t* data, const uint64_t* offs, uint64_t n, uint8_t out[32]);
int or_struct_roots(const uint8_t* rec, uint64_t n, uint32_t rec_len, const uint32_t* kind,
                    const uint32_t* off, const uint32_t* len, uint32_t nf, uint8_t* roots, int nthreads);

#endif
