/* spgg_test.h -- TEST-ONLY entry points of libspgg_hip.so.
 *
 * Not part of the product ABI (spgg_abi.h): no production caller needs them, and a binding
 * for the reference never declares them.  The GPU tests use them to drive
 * failure paths that a healthy device never takes.
 */
#ifndef SPGG_TEST_H
#define SPGG_TEST_H

#include "spgg_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* OR flags (SPGG_GEN_ERR_* bits) into the context's error word on the generator's stream,
 * as an exhausted bounded wait does (MT19937 contexts): spgg_status / spgg_flush then report
 * it (tests/test_gpu_pipeline.py). */
int spgg_test_set_error(spgg_ctx* ctx, uint32_t flags);

#ifdef __cplusplus
}
#endif
#endif /* SPGG_TEST_H */
