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
 *      (row axis, row 0, position 1);
 *   4. a resident square (cda_square_create, the proof / GetCommitment
 *      cache): its DAH equals the golden k = 2 root, the subtree root of the
 *      empty walk is row root 0, the walk [WalkLeft] is the standalone
 *      erasured tree over row 0's two ODS cells (cda_nmt_axis_root), a walk
 *      below the leaves fails with the cache's text;
 *   5. rsmt2d Codec.Encode / Decode (cda_rs_encode / cda_rs_decode): 8 data
 *      shards, half of data + parity erased, reconstructed bit-exactly;
 *   6. Repair (cda_repair) of the k = 2 EDS with Q0 erased: the EDS back.
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

    /* 4. resident square of the k = 2 constant shares */
    {
        uint8_t ods2[4 * 512], r0[90], sub[90], want[90], dr[32], rr[4 * 90];
        char got[65];
        uint32_t kk = 0;
        cda_square* sq = NULL;
        constant_shares(ods2, 4);
        if (cda_square_create(ctx, ods2, 4, &sq) != CDA_OK) return fail("cda_square_create");
        if (cda_square_dah(sq, &kk, rr, NULL, dr, NULL) != CDA_OK || kk != 2) return fail("cda_square_dah");
        hex(dr, 32, got);
        if (strcmp(got, golden_k2)) return fail("resident square data root");
        if (cda_square_subtree_root(sq, 0, NULL, 0, r0) != CDA_OK || memcmp(r0, rr, 90))
            return fail("subtree root of the empty walk");
        const uint8_t left[1] = {0};
        if (cda_square_subtree_root(sq, 0, left, 1, sub) != CDA_OK) return fail("subtree root [WalkLeft]");
        if (cda_nmt_axis_root(ctx, ods2, 512, 2, 2, 0, want) != CDA_OK || memcmp(sub, want, 90))
            return fail("subtree root [WalkLeft] vs the standalone tree");
        const uint8_t deep[3] = {0, 0, 0};
        if (cda_square_subtree_root(sq, 0, deep, 3, sub) != CDA_ERR_INVALID ||
            !strstr(cda_last_error(ctx), "did not find sub tree root"))
            return fail("walk below the leaves");
        cda_square_destroy(sq);
    }

    /* 5. Codec.Encode / Decode: 8 data shards of 64 B, half of the 16 lost */
    {
        uint8_t shards[16 * 64], keep[16 * 64], present[16];
        for (int i = 0; i < 8 * 64; i++) shards[i] = (uint8_t)(i * 37 + 11);
        if (cda_rs_encode(ctx, shards, 8, 64, 1, shards + 8 * 64) != CDA_OK) return fail("cda_rs_encode");
        memcpy(keep, shards, sizeof keep);
        for (int i = 0; i < 16; i++) {
            present[i] = (i % 2 == 0);
            if (!present[i]) memset(shards + i * 64, 0xA5, 64);
        }
        if (cda_rs_decode(ctx, shards, present, 8, 64, 1) != CDA_OK) return fail("cda_rs_decode");
        if (memcmp(shards, keep, sizeof keep)) return fail("decoded shards");
        memset(present, 0, 9);   /* 7 of 16 left */
        if (cda_rs_decode(ctx, shards, present, 8, 64, 1) != CDA_ERR_UNREPAIRABLE) return fail("too few shards");
    }

    /* 6. Repair of the k = 2 EDS with Q0 erased */
    {
        uint8_t ods2[4 * 512], eds2[16 * 512], keep[16 * 512], rr[4 * 90], cr[4 * 90], dr[32], present[16];
        int32_t byz_axis = -1;
        uint32_t byz_index = 0;
        constant_shares(ods2, 4);
        ods2[29] = 0x07;   /* not all cells equal */
        if (cda_extend_dah(ctx, ods2, 4, eds2, rr, cr, dr) != CDA_OK) return fail("extend for repair");
        memcpy(keep, eds2, sizeof keep);
        for (int i = 0; i < 16; i++) {
            present[i] = !((i / 4) < 2 && (i % 4) < 2);
            if (!present[i]) memset(eds2 + i * 512, 0, 512);
        }
        if (cda_repair(ctx, eds2, present, 4, rr, cr, &byz_axis, &byz_index) != CDA_OK) return fail("cda_repair");
        if (memcmp(eds2, keep, sizeof keep)) return fail("repaired EDS");
    }

    cda_ctx_destroy(ctx);
    printf("c host ok: %s\n", cda_version());
    return 0;
}
