/* TEST INFRASTRUCTURE ONLY — see farmhash32.c header. */
#ifndef RINGPOP_ORACLE_FARMHASH32_H
#define RINGPOP_ORACLE_FARMHASH32_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
uint32_t oracle_farmhash32(const uint8_t *s, size_t len);
uint32_t oracle_farmhash32_seed(const uint8_t *s, size_t len, uint32_t seed);
uint32_t oracle_farmhash_test_seed(int offset, int salt);
void oracle_farmhash32_batch(const uint8_t *bytes, const uint64_t *offsets, size_t n, uint32_t *out);
#ifdef __cplusplus
}
#endif
#endif
