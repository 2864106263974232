/*
 * cda_host_smoke.c -- libcda.so driven from plain C, the way the cgo package of
 * INTEGRATION.md section 2 drives it (no Python, no torch in the process; the
 * C compiler sees only include/cda.h, as cgo's does).
 *
 * Checks, each against the reference's own expectations:
 *   1. cda_extend_dah on the constant shares of
 *      pkg/da/data_availability_header_test.go:247-263 (generateShares) at
 *      k = 2 and k = 128: the data roots of TestNewDataAvailabilityHeader
 *      (:34-68);
 *   2. cda_extend_shares on 5 shares: CDA_ERR_NOT_POW2 with the reference's
 *      text "number of shares is not a power of 2: got 5" (:68);
 *   3. cda_dah_from_eds on an EDS whose Q0 row 0 is out of namespace order:
 *      CDA_ERR_PUSH_ORDER, the nmt message, and cda_push_order_detail =
 *      (row axis, row 0, position 1).
 * Prints "c host ok" and exits 0, or names the failed check and exits 1.
 * Build: gcc -std=c11 -I include tests/c_host/cda_host_smoke.c
 *        -L celestia-app_amd -lcda -Wl,-rpath,<abs celestia-app_amd>
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cda.h"

static const char* golden_k2 = "b56e4d251ac266f4b91cc5464b3fc7efcbdc888064647496d13133f0dc65ac25";
static const char* golden_k128 = "0bd3abeeacfbb0b92dfbdac4a154868e3c4e79666f7fcf6c620bb90dd3a0dcf0";

static void constant_shares(uint8_t* out, uint32_t count) {
    for (uint32_t i = 0; i < count; i++) {
        uint8_t* s = out + (size_t)i * 512;
        memset(s, 0, 19);            /* version 0, 18 zero bytes */
        memset(s + 19, 0x01, 10);    /* MustNewV0(bytes.Repeat([]byte{1}, 10)) */
        memset(s + 29, 0xFF, 483);
    }
}

static void hex(const uint8_t* b, size_t n, char* out) {
    for (size_t i = 0; i < n; i++) sprintf(out + 2 * i, "%02x", b[i]);
}

static int fail(const char* what) {
    fprintf(stderr, "c host FAILED: %s\n", what);
    return 1;
}

static int check_root(cda_ctx* ctx, uint32_t k, const char* want) {
    const uint32_t W = 2 * k;
    uint8_t* ods = malloc((size_t)k * k * 512);
    uint8_t* eds = malloc((size_t)W * W * 512);
    uint8_t* rows = malloc((size_t)W * 90);
    uint8_t* cols = malloc((size_t)W * 90);
    uint8_t root[32];
    char got[65];
    if (!ods || !eds || !rows || !cols) return fail("malloc");
    constant_shares(ods, k * k);
    int rc = cda_extend_dah(ctx, ods, k * k, eds, rows, cols, root);
    if (rc != CDA_OK) {
        fprintf(stderr, "cda_extend_dah k=%u: %d %s\n", k, rc, cda_last_error(ctx));
        return fail("cda_extend_dah");
    }
    hex(root, 32, got);
    /* Q0 of the returned EDS is the input, row-major in the 2k-wide layout */
    for (uint32_t r = 0; r < k; r++)
        if (memcmp(eds + (size_t)r * W * 512, ods + (size_t)r * k * 512, (size_t)k * 512)) return fail("EDS Q0");
    free(ods);
    free(eds);
    free(rows);
    free(cols);
    if (strcmp(got, want)) {
        fprintf(stderr, "k=%u data root %s, want %s\n", k, got, want);
        return fail("golden data root");
    }
    return 0;
}

int main(void) {
    cda_ctx* ctx = NULL;
    int rc = cda_ctx_create(-1, &ctx);
    if (rc != CDA_OK) return fail("cda_ctx_create");
    if (check_root(ctx, 2, golden_k2) || check_root(ctx, 128, golden_k128)) return 1;

    /* 2. ExtendShares on a non-square share count */
    uint8_t five[5 * 512];
    uint8_t eds5[16 * 512];
    constant_shares(five, 5);
    rc = cda_extend_shares(ctx, five, 5, eds5);
    if (rc != CDA_ERR_NOT_POW2) return fail("non-power-of-2 code");
    if (!strstr(cda_last_error(ctx), "number of shares is not a power of 2: got 5")) return fail("non-power-of-2 text");

    /* 3. roots of an EDS whose Q0 row 0 pushes namespace 0x...02 before 0x...01 */
    const uint32_t k = 4, W = 8;
    uint8_t ods[16 * 512];
    static uint8_t eds[64 * 512];
    uint8_t rows[8 * 90], cols[8 * 90], root[32];
    constant_shares(ods, 16);
    ods[28] = 0x02;   /* cell (0, 0) gets the larger namespace */
    rc = cda_extend_shares(ctx, ods, 16, eds);
    if (rc != CDA_OK) return fail("cda_extend_shares");   /* ExtendShares never hashes */
    rc = cda_dah_from_eds(ctx, eds, W, rows, cols, root);
    if (rc != CDA_ERR_PUSH_ORDER) return fail("push-order code");
    if (!strstr(cda_last_error(ctx), "pushed data has to be lexicographically ordered by namespace IDs"))
        return fail("push-order text");
    int32_t axis = -1;
    uint32_t index = 99, position = 99;
    cda_push_order_detail(ctx, &axis, &index, &position);
    if (axis != 0 || index != 0 || position != 1) return fail("push-order detail");
    (void)k;

    cda_ctx_destroy(ctx);
    printf("c host ok: %s\n", cda_version());
    return 0;
}
