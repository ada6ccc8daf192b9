// kp_out.h -- the long output table's rows (host code): SURVEY.md §8(f) row 3.
//
// With -l the reference prints one row per k-mer of every pattern of the partition
// (src/kmerpapa/cli.py:301-316):  f"{context} {c_neg} {c_pos} {c_rate} {pattern} {p_neg}
// {p_pos} {p_rate}", c_rate = float(c_pos) / (c_pos + c_neg).  At 9- and 11-mer scale that
// is 131,072+ rows of Python string formatting; here the per-k-mer part of every row is
// formatted natively and the per-pattern tail (" pattern p_neg p_pos p_rate\n", a few
// thousand of them) comes formatted from the caller.
//
// Floats are written as Python's repr() writes them (float_repr_style 'short',
// Python/pystrtod.c format_float_short with mode 'r' and Py_DTSF_ADD_DOT_0): the shortest
// digit string that reads back to the same double (std::to_chars, correctly rounded like
// Python's dtoa mode 0), in positional notation when the decimal point position decpt
// (value = 0.d1d2... x 10^decpt) satisfies -4 < decpt <= 16, otherwise as d.ddde[+-]XX.
#pragma once
#include <stdint.h>
#include <string.h>

#include <charconv>
#include <cmath>

namespace kpout {

// Python repr of a finite or special double; returns the number of chars written (<= 32)
inline int py_repr(double x, char *out) {
    if (std::isnan(x)) {
        memcpy(out, "nan", 3);
        return 3;
    }
    int n = 0;
    if (std::signbit(x)) out[n++] = '-';
    const double a = std::fabs(x);
    if (std::isinf(a)) {
        memcpy(out + n, "inf", 3);
        return n + 3;
    }
    if (a == 0.0) {
        memcpy(out + n, "0.0", 3);
        return n + 3;
    }
    char sci[40];
    const auto r = std::to_chars(sci, sci + sizeof(sci), a, std::chars_format::scientific);  // d[.ddd]e[+-]XX
    const char *e = static_cast<const char *>(memchr(sci, 'e', (size_t)(r.ptr - sci)));
    char dig[24];
    int nd = 0;
    for (const char *q = sci; q < e; ++q)
        if (*q != '.') dig[nd++] = *q;
    int ex = 0;
    {
        const char *q = e + 1;
        const bool neg = *q == '-';
        if (*q == '+' || *q == '-') ++q;
        for (; q < r.ptr; ++q) ex = 10 * ex + (*q - '0');
        if (neg) ex = -ex;
    }
    const int decpt = ex + 1;
    if (decpt <= -4 || decpt > 16) {  // exponent notation: d[.ddd]e-XX, exponent >= 2 digits
        out[n++] = dig[0];
        if (nd > 1) {
            out[n++] = '.';
            memcpy(out + n, dig + 1, (size_t)(nd - 1));
            n += nd - 1;
        }
        out[n++] = 'e';
        out[n++] = ex < 0 ? '-' : '+';
        const int ax = ex < 0 ? -ex : ex;
        if (ax >= 100) out[n++] = (char)('0' + ax / 100);
        out[n++] = (char)('0' + (ax / 10) % 10);
        out[n++] = (char)('0' + ax % 10);
        return n;
    }
    if (decpt <= 0) {  // 0.000ddd
        out[n++] = '0';
        out[n++] = '.';
        for (int i = 0; i < -decpt; ++i) out[n++] = '0';
        memcpy(out + n, dig, (size_t)nd);
        return n + nd;
    }
    if (decpt >= nd) {  // ddd000.0
        memcpy(out + n, dig, (size_t)nd);
        n += nd;
        for (int i = nd; i < decpt; ++i) out[n++] = '0';
        out[n++] = '.';
        out[n++] = '0';
        return n;
    }
    memcpy(out + n, dig, (size_t)decpt);  // dd.ddd
    n += decpt;
    out[n++] = '.';
    memcpy(out + n, dig + decpt, (size_t)(nd - decpt));
    return n + nd - decpt;
}

inline int put_i64(int64_t v, char *out) {
    const auto r = std::to_chars(out, out + 24, v);
    return (int)(r.ptr - out);
}

// Rows "kmer c_neg c_pos c_rate" + tails[pid[i]] for i < n.  kmers: n * k letters;
// tail t = tails[tail_off[t] .. tail_off[t + 1]).  Returns bytes written, or -1 if cap is
// too small, -2 if a row has c_pos + c_neg == 0 (Python raises ZeroDivisionError there),
// -3 for a pattern index out of range.
inline int64_t long_rows(const char *kmers, int k, const int64_t *c_neg, const int64_t *c_pos, const uint32_t *pid,
                         uint64_t n, const char *tails, const uint64_t *tail_off, uint64_t n_tails, char *out,
                         uint64_t cap) {
    uint64_t w = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (pid[i] >= n_tails) return -3;
        const int64_t tot = c_pos[i] + c_neg[i];
        if (tot == 0) return -2;
        const uint64_t tl = tail_off[pid[i] + 1] - tail_off[pid[i]];
        if (w + (uint64_t)k + 3 * 32 + tl > cap) return -1;
        memcpy(out + w, kmers + i * (uint64_t)k, (size_t)k);
        w += (uint64_t)k;
        out[w++] = ' ';
        w += (uint64_t)put_i64(c_neg[i], out + w);
        out[w++] = ' ';
        w += (uint64_t)put_i64(c_pos[i], out + w);
        out[w++] = ' ';
        w += (uint64_t)py_repr((double)c_pos[i] / (double)tot, out + w);
        memcpy(out + w, tails + tail_off[pid[i]], (size_t)tl);
        w += tl;
    }
    return (int64_t)w;
}

}  // namespace kpout
