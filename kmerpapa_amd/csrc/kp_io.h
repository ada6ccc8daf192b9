// kp_io.h -- k-mer count file parser (host code): SURVEY.md §8(f) row 1.
//
// Reads the reference's two input formats into sorted 2-bit k-mer codes (first letter
// most significant, so code order = the reference's sorted-context order) with counts:
//
//   "kmer count" lines            src/kmerpapa/io_utils.py read_dict :82-136
//     (counts of equal k-mers summed; optional down-sizing to the central `length`
//      letters, :50-79; optional super-pattern filter)
//   "kmer positive background"    read_joint_kmer_counts :3-46
//     (the last line of a k-mer wins, totals sum every line; background >= positive)
//
// Line and token rules follow Python's text-mode file iteration and str.split(): lines
// end at \n, \r or \r\n; tokens are runs of non-whitespace; a line with the wrong number
// of tokens is an error (the reference's tuple unpacking); lines whose k-mer has a letter
// other than A/C/G/T are skipped before the counts are parsed.  A count is Python's
// int(tok), or int(float(tok)) when that fails (truncation toward zero).
//
// Deliberate difference: every k-mer of one file must have the same length (the
// reference would silently slice mixed lengths into keys of different lengths, which
// its later steps cannot use); such a file is an input error here.
#pragma once
#include <ctype.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

namespace kpio {

struct table {
    int k = 0;
    std::vector<uint64_t> code;  // sorted, unique
    std::vector<int64_t> c0, c1; // per code: count (2 columns) / positive, background - positive (3 columns)
    int64_t total0 = 0, total1 = 0;
};

inline bool is_space(unsigned char c) {  // str.isspace() for ASCII
    return c == ' ' || (c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x1f);
}

inline int base2(unsigned char c) {
    switch (c) {
        case 'A': return 0;
        case 'C': return 1;
        case 'G': return 2;
        case 'T': return 3;
        default: return -1;
    }
}

// IUPAC letter -> mask of A/C/G/T (bit b = base b); 0 for anything else
inline unsigned iupac_mask(char c) {
    switch (c) {
        case 'A': return 1; case 'C': return 2; case 'G': return 4; case 'T': return 8;
        case 'R': return 1 | 4; case 'Y': return 2 | 8; case 'S': return 2 | 4; case 'W': return 1 | 8;
        case 'K': return 4 | 8; case 'M': return 1 | 2; case 'B': return 2 | 4 | 8; case 'D': return 1 | 4 | 8;
        case 'H': return 1 | 2 | 8; case 'V': return 1 | 2 | 4; case 'N': return 15;
        default: return 0;
    }
}

inline std::string quoted(const char *s, size_t n) { return "'" + std::string(s, n) + "'"; }

// digits with single underscores between them (Python's int()/float() digit groups);
// appends the digits to out
inline bool digit_part(const char *&p, const char *e, std::string &out) {
    if (p == e || *p < '0' || *p > '9') return false;
    out.push_back(*p++);
    while (p < e) {
        if (*p >= '0' && *p <= '9') {
            out.push_back(*p++);
        } else if (*p == '_' && p + 1 < e && p[1] >= '0' && p[1] <= '9') {
            ++p;
        } else {
            break;
        }
    }
    return true;
}

// Python int(tok), else int(float(tok)).  Returns "" or an error text.
inline std::string parse_count(const char *s, size_t n, int64_t *v) {
    const char *p = s, *e = s + n;
    bool neg = false;
    if (p < e && (*p == '+' || *p == '-')) neg = (*p++ == '-');
    std::string d;
    const char *q = p;
    if (digit_part(q, e, d) && q == e) {  // int(tok)
        unsigned long long x = 0;
        for (char c : d) {
            if (x > (0x7FFFFFFFFFFFFFFFull - (uint64_t)(c - '0')) / 10) return "count too large: " + quoted(s, n);
            x = x * 10 + (uint64_t)(c - '0');
        }
        *v = neg ? -(int64_t)x : (int64_t)x;
        return "";
    }
    // float(tok): [sign] (inf | infinity | nan | digits[.digits][exp] | .digits[exp])
    std::string lower(p, e);
    for (char &c : lower) c = (char)tolower((unsigned char)c);
    if (lower == "inf" || lower == "infinity") return "cannot convert float infinity to integer";
    if (lower == "nan") return "cannot convert float NaN to integer";
    std::string num = neg ? "-" : "";
    q = p;
    bool mant = digit_part(q, e, num);
    if (q < e && *q == '.') {
        num.push_back('.');
        ++q;
        std::string frac;
        if (digit_part(q, e, frac)) {
            num += frac;
            mant = true;
        }
    }
    if (mant && q < e && (*q == 'e' || *q == 'E')) {
        num.push_back('e');
        ++q;
        if (q < e && (*q == '+' || *q == '-')) num.push_back(*q++);
        if (!digit_part(q, e, num)) mant = false;
    }
    if (!mant || q != e) return "could not convert string to float: " + quoted(s, n);
    const double f = strtod(num.c_str(), nullptr);
    if (std::isinf(f)) return "cannot convert float infinity to integer";
    const double t = trunc(f);
    if (!(fabs(t) < 9.2e18)) return "count too large: " + quoted(s, n);
    *v = (int64_t)t;
    return "";
}

struct rec {
    uint64_t code;
    uint64_t seq;  // line order (the last line of a k-mer wins in the 3-column format)
    int64_t a, b;
};

// columns = 2 or 3; super_pattern may be null/empty; length > 0 only for 2 columns.
inline std::string parse(const char *text, uint64_t nbytes, int columns, const char *super_pattern, int length,
                         table &T) {
    T = table();
    if (columns != 2 && columns != 3) return "columns must be 2 or 3";
    const std::string sp = super_pattern ? super_pattern : "";
    if (columns == 2 && length <= 0 && !sp.empty()) length = (int)sp.size();  // read_dict :93-94
    std::vector<rec> recs;
    const char *p = text, *end = text + nbytes;
    int width = -1;          // letters of the file's k-mers
    size_t lo = 0, hi = 0;   // kept window (2 columns)
    uint64_t seq = 0;
    while (p < end) {
        const char *ls = p;
        while (p < end && *p != '\n' && *p != '\r') ++p;
        const char *le = p;
        if (p < end) {
            if (*p == '\r' && p + 1 < end && p[1] == '\n') ++p;
            ++p;
        }
        // tokens
        const char *tok[3];
        size_t tlen[3];
        int nt = 0;
        for (const char *q = ls; q < le;) {
            while (q < le && is_space((unsigned char)*q)) ++q;
            if (q >= le) break;
            const char *ts = q;
            while (q < le && !is_space((unsigned char)*q)) ++q;
            if (nt < columns) {
                tok[nt] = ts;
                tlen[nt] = (size_t)(q - ts);
            }
            ++nt;
        }
        if (nt > columns) return "too many values to unpack (expected " + std::to_string(columns) + ")";
        if (nt < columns)
            return "not enough values to unpack (expected " + std::to_string(columns) + ", got " + std::to_string(nt) +
                   ")";
        bool nuc = true;
        for (size_t i = 0; i < tlen[0]; ++i) nuc = nuc && base2((unsigned char)tok[0][i]) >= 0;
        if (!nuc) continue;  // not set(kmer) <= {A,C,G,T}
        rec r;
        r.seq = seq++;
        r.b = 0;
        if (columns == 2) {  // count first, as read_dict :101-103
            std::string err = parse_count(tok[1], tlen[1], &r.a);
            if (!err.empty()) return err;
            if (r.a < 0) return "negative counts are not allowed, bad line:\n" + std::string(ls, le);
        }
        if (width < 0) {
            width = (int)tlen[0];
            lo = 0;
            hi = (size_t)width;
            if (columns == 2 && length > 0 && length != width) {
                if (width <= length)
                    return "k-mer:" + std::string(tok[0], tlen[0]) + " cannot be reduced to length " +
                           std::to_string(length);
                lo = (size_t)(width / 2 - length / 2);
                hi = lo + (size_t)length;
            }
            if (hi - lo > 32) return "k-mers longer than 32 letters are not supported";
        } else if ((int)tlen[0] != width) {
            return "k-mers of different lengths in one file (" + std::to_string(width) + " and " +
                   std::to_string(tlen[0]) + ")";
        }
        const char *kmer = tok[0] + lo;
        const size_t kl = hi - lo;
        if (columns == 2) {
            if (!sp.empty()) {
                if (sp.size() != kl) return "super pattern length " + std::to_string(sp.size()) +
                                            " != k-mer length " + std::to_string(kl);
                bool in = true;
                for (size_t i = 0; i < kl && in; ++i) in = (iupac_mask(sp[i]) >> base2((unsigned char)kmer[i])) & 1u;
                if (!in) continue;
            }
            T.total0 += r.a;
        } else {
            int64_t bg = 0, pos = 0;
            std::string err = parse_count(tok[2], tlen[2], &bg);
            if (err.empty()) err = parse_count(tok[1], tlen[1], &pos);
            if (!err.empty()) return err;
            if (bg - pos < 0)
                return "background counts should be larger than the positive counts so that a negative set can be "
                       "created by subtraction the positive count from the background count. Problematic kmer: " +
                       std::string(tok[0], tlen[0]);
            if (!sp.empty()) {  // Pattern.__contains__ compares zip(pattern, kmer)
                bool in = true;
                for (size_t i = 0; i < kl && i < sp.size() && in; ++i)
                    in = (iupac_mask(sp[i]) >> base2((unsigned char)kmer[i])) & 1u;
                if (!in) continue;
            }
            T.total0 += bg;   // n_sites
            T.total1 += pos;  // n_pos
            r.a = pos;
            r.b = bg - pos;
        }
        uint64_t c = 0;
        for (size_t i = 0; i < kl; ++i) c = (c << 2) | (uint64_t)base2((unsigned char)kmer[i]);
        r.code = c;
        recs.push_back(r);
    }
    T.k = width < 0 ? 0 : (int)(hi - lo);
    std::sort(recs.begin(), recs.end(),
              [](const rec &x, const rec &y) { return x.code != y.code ? x.code < y.code : x.seq < y.seq; });
    for (size_t i = 0; i < recs.size();) {
        size_t j = i;
        int64_t a = 0;
        while (j < recs.size() && recs[j].code == recs[i].code) a += recs[j++].a;
        T.code.push_back(recs[i].code);
        if (columns == 2) {
            T.c0.push_back(a);
            T.c1.push_back(0);
        } else {  // last line wins
            T.c0.push_back(recs[j - 1].a);
            T.c1.push_back(recs[j - 1].b);
        }
        i = j;
    }
    if (columns == 3) {
        const int64_t n_sites = T.total0, n_pos = T.total1;
        T.total0 = n_sites - n_pos;  // n_negative_total
        T.total1 = n_pos;
    }
    return "";
}

}  // namespace kpio
