// CPU check of drl::qnet_pack_elem (the learner's parameter -> packed element
// map) against drl::qnet_pack_slot (drl_qnet_pack's element -> parameter map):
// every weight of every layer, and a code net's layer-0 bias, round-trips, and
// the forward map hits each real weight exactly once.  Built and run by
// tests/test_pack_index.py (host code only).
#include <stdio.h>

#include <vector>

#include "../../dronerl_amd/csrc/dronerl_internal.h"

static int check(int in0, const int* hidden, int nh, int code_w) {
    int in[4], out[4], kt[4];
    const int L = nh + 1;
    for (int l = 0; l < L; ++l) {
        in[l] = l == 0 ? in0 : hidden[l - 1];
        out[l] = l < nh ? hidden[l] : 5;
        kt[l] = l == 0 ? (code_w ? drl::lay::code_kt(code_w) : ((in0 + 31) / 32 + DRL_QN_RING - 1) / DRL_QN_RING * DRL_QN_RING)
                       : in[l] / 32;
    }
    int bad = 0;
    for (int l = 0; l < L; ++l) {
        const int nt = (out[l] + 15) / 16;
        const int64_t n = (int64_t)nt * kt[l] * 512;
        std::vector<int> hits((size_t)out[l] * in[l], 0), bias_hits(out[l], 0);
        for (int64_t e = 0; e < n; ++e) {
            const drl::PackSlot s = drl::qnet_pack_slot(l, e, kt[l], code_w, in[l]);
            if (s.row >= out[l]) continue;
            if (s.k < 0) {
                if (l != 0 || !code_w) ++bad;
                else {
                    bias_hits[s.row]++;
                    if (drl::qnet_pack_elem(0, s.row, -1, kt[0], code_w) != e) ++bad;
                }
                continue;
            }
            if (s.k >= in[l]) continue;
            hits[(size_t)s.row * in[l] + s.k]++;
            if (drl::qnet_pack_elem(l, s.row, s.k, kt[l], code_w) != e) ++bad;
        }
        for (int h : hits) bad += h != 1;
        if (l == 0 && code_w)
            for (int h : bias_hits) bad += h != 1;
    }
    return bad;
}

int main() {
    const int h1[] = {128, 64}, h2[] = {96, 32, 32}, h3[] = {64}, h4[] = {128, 128, 128}, h5[] = {32, 32};
    struct Case { int in0; const int* h; int nh; int code_w; } cases[] = {
        {294, h1, 2, 7}, {294, h1, 2, 0}, {150, h2, 3, 5}, {486, h3, 1, 9}, {294, h4, 3, 7}, {150, h5, 2, 0},
        {486, h1, 2, 9}, {30, h3, 1, 0}};
    int total = 0;
    for (const Case& c : cases) {
        const int b = check(c.in0, c.h, c.nh, c.code_w);
        printf("in %d hidden %d code_w %d: %d bad\n", c.in0, c.h[0], c.code_w, b);
        total += b;
    }
    printf(total ? "FAIL\n" : "OK\n");
    return total ? 1 : 0;
}
