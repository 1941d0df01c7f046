// Text matrix/vector I/O with the reference's file contract (src/matr_utils.c:9-83):
//   <dir>/matrix_<R>_<C>.txt   (build_matrix_filename, matr_utils.c:9-12)
//   <dir>/vector_<n>.txt       (build_vector_filename, matr_utils.c:15-18)
// whitespace-separated tokens read row-major with "%lf" (matr_utils.c:55-59, 78-80).
//
// The reference parses with one fscanf per value; at 16384^2 and up (1.9-120 GB of text)
// that is impractical, so here the file is mmap'd, split into per-thread ranges on
// whitespace boundaries, tokens are counted, prefix-summed, then converted exactly as strtod
// (the conversion fscanf("%lf") performs) would: Clinger's exact fast path for short decimal
// tokens (parse_fast), strtod itself for the rest, so the doubles are bit-identical to the
// reference's.
// Differences, all deliberate: 64-bit indices; a file with fewer tokens than R*C is an error
// (the reference ignores fscanf's return and leaves garbage); the file is closed.
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <string>
#include <vector>

#include "common.h"

using namespace mvg;

namespace {

inline bool is_space(char c) {
    return c == ' ' || c == '\n' || c == '\t' || c == '\r' || c == '\v' || c == '\f';
}
// the same test as 0/1 arithmetic ('\t' ... '\r' are 9 ... 13)
inline unsigned is_space_bits(char c) {
    const unsigned u = (unsigned char)c;
    return (unsigned)(u == 32u) | (unsigned)(u - 9u < 5u);
}

constexpr double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                               1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// Decimal token -> double without strtod for the common case, Clinger's fast path: a token
// [+-]digits[.digits][(e|E)[+-]digits] whose significant digits (leading and trailing zeros
// dropped) form an integer m <= 2^53 and whose decimal exponent e lies in [-22, 22]. Then m and
// 10^|e| are exact doubles and one IEEE multiply or divide rounds the exact value once, to
// nearest — the double strtod (correctly rounded) returns. The reference's inputs ("%.4f",
// README.md:32) always take this path; anything else (more digits, hex, inf/nan, a malformed
// token) returns false and the caller falls back to strtod, so results never differ from it.
inline bool parse_fast(const char* p, const char* end, double* out) {
    bool neg = false;
    if (p < end && (*p == '+' || *p == '-')) neg = *p++ == '-';
    uint64_t m = 0;
    int nd = 0;     // digits in m (from the first nonzero digit on)
    int zeros = 0;  // zeros seen since the last nonzero digit, not yet folded into m
    int e10 = 0;
    bool any = false, dot = false;
    for (; p < end; ++p) {
        const char c = *p;
        if (c >= '0' && c <= '9') {
            any = true;
            if (dot) --e10;
            if (c == '0') {
                if (nd) ++zeros;
                continue;
            }
            for (; zeros > 0; --zeros, ++nd) {
                if (nd >= 19) return false;
                m *= 10;
            }
            if (nd >= 19) return false;
            m = m * 10 + (uint64_t)(c - '0');
            ++nd;
        } else if (c == '.' && !dot) {
            dot = true;
        } else {
            break;
        }
    }
    if (!any) return false;
    e10 += zeros;  // trailing zeros: m * 10^zeros
    if (p < end) {
        if (*p != 'e' && *p != 'E') return false;
        ++p;
        bool eneg = false;
        if (p < end && (*p == '+' || *p == '-')) eneg = *p++ == '-';
        if (p >= end) return false;
        int ex = 0;
        for (; p < end; ++p) {
            if (*p < '0' || *p > '9') return false;
            if (ex < 100000) ex = ex * 10 + (*p - '0');
        }
        e10 += eneg ? -ex : ex;
    }
    if (m == 0) {
        *out = neg ? -0.0 : 0.0;
        return true;
    }
    if (m > (1ull << 53) || e10 < -22 || e10 > 22) return false;
    const double v = e10 < 0 ? (double)m / kPow10[-e10] : (double)m * kPow10[e10];
    *out = neg ? -v : v;
    return true;
}

// The reference's own token shape, [-]digits[.digits] with at most 15 digits in all (its inputs
// are "%.4f"): m < 10^15 < 2^53 and 10^f (f <= 15 fraction digits) are exact doubles, so
// m / 10^f is strtod's correctly rounded result — the same double parse_fast gives, which strips
// zeros first (the rational m / 10^f is the same either way). Leading zeros count as digits
// here, which only makes the check stricter. The fraction is read 8 bytes at a time (SWAR):
// the bytes that are digits are found with one add and mask, and up to 8 of them are converted
// with three multiplies. p points at the token's first byte; returns the byte after the token,
// or nullptr (nothing written) for any other shape, or when fewer than 8 bytes follow the
// point (the caller's general path handles the file's last bytes).
inline const char* parse_plain(const char* p, const char* end, double* out) {
    const bool neg = *p == '-';
    p += neg;
    uint64_t m = 0;
    int nd = 0;
    for (; p < end; ++p) {
        const unsigned d = (unsigned)(unsigned char)*p - '0';
        if (d >= 10) break;
        m = m * 10 + d;
        ++nd;
    }
    int nf = 0;
    if (p < end && *p == '.') {
        ++p;
        if (end - p < 8) return nullptr;
        uint64_t w;
        memcpy(&w, p, 8);
        const uint64_t a = w ^ 0x3030303030303030ull;  // digit bytes -> 0 ... 9
        const uint64_t nondigit = ((((a & 0x7F7F7F7F7F7F7F7Full) + 0x7676767676767676ull) | a) &
                                   0x8080808080808080ull);
        if (nondigit == 0) return nullptr;  // 8 or more fraction digits: the general path
        nf = __builtin_ctzll(nondigit) >> 3;
        if (nf > 0) {
            uint64_t v = a << (8 * (8 - nf));  // digits into the top bytes, zeros before them
            v = ((v & 0x0F0F0F0F0F0F0F0Full) * 2561) >> 8;
            v = ((v & 0x00FF00FF00FF00FFull) * 6553601) >> 16;
            v = ((v & 0x0000FFFF0000FFFFull) * 42949672960001ull) >> 32;
            m = m * (uint64_t)kPow10[nf] + v;
            nd += nf;
        }
        p += nf;
    }
    if (nd == 0 || nd > 15 || (p < end && !is_space(*p))) return nullptr;
    const double v = nf > 0 ? (double)(int64_t)m / kPow10[nf] : (double)(int64_t)m;  // m < 10^15
    *out = neg ? -v : v;
    return p;
}

// The two per-thread loops are built for AVX-512BW and AVX2 beside the baseline x86-64 and
// picked at load time (the library is built here and runs on the GPU box's host).
#define MVG_CPU_CLONES __attribute__((target_clones("avx512bw", "avx2", "default")))

// Tokens in [p, end): a token starts where a non-space follows a space (or at p: every range
// but the first starts on whitespace). Branch-free over bytes, so the loop vectorises.
MVG_CPU_CLONES int64_t count_tokens(const char* p, const char* end) {
    if (p >= end) return 0;
    const unsigned char* b = (const unsigned char*)p;
    const size_t len = (size_t)(end - p);
    uint64_t k = !is_space(p[0]);
    for (size_t i = 1; i < len; ++i) k += is_space_bits((char)b[i - 1]) & ~is_space_bits((char)b[i]) & 1u;
    return (int64_t)k;
}

// One token of [p, end) into *out (p at the token's first byte); returns the byte after it.
// Sets *bad if the token is not a number.
inline const char* parse_token(const char* p, const char* end, double* out, int* bad) {
    if (const char* q = parse_plain(p, end, out)) return q;
    const char* j = p;
    while (j < end && !is_space(*j)) ++j;
    const size_t tl = (size_t)(j - p);
    char buf[128];
    if (parse_fast(p, j, out)) {
        // exact: the value strtod would return
    } else if (tl < sizeof(buf)) {
        memcpy(buf, p, tl);
        buf[tl] = '\0';
        char* ep = nullptr;
        *out = strtod(buf, &ep);
        *bad |= ep == buf;
    } else {
        std::string tok(p, tl);
        char* ep = nullptr;
        *out = strtod(tok.c_str(), &ep);
        *bad |= ep == tok.c_str();
    }
    return j;
}

// kStreams consecutive ranges [p[s], end[s]) into out[k0[s] ...], stopping at out[n - 1], one
// token of each in turn: a token's end (hence the next one's address) depends on the bytes just
// parsed, so one range alone is a chain of dependent loads; four interleaved chains keep the
// core busy. Returns 1 if a token is not a number, else 0.
constexpr int kStreams = 4;
MVG_CPU_CLONES int parse_ranges(const char* const* p0, const char* const* end, const int64_t* k0, int64_t n,
                                double* out) {
    const char* p[kStreams];
    int64_t k[kStreams];
    for (int s = 0; s < kStreams; ++s) p[s] = p0[s], k[s] = k0[s];
    int bad = 0;
    for (;;) {
        bool any = false;
        for (int s = 0; s < kStreams; ++s) {
            while (p[s] < end[s] && is_space(*p[s])) ++p[s];
            if (p[s] >= end[s] || k[s] >= n) continue;
            any = true;
            p[s] = parse_token(p[s], end[s], &out[k[s]], &bad);
            ++k[s];
        }
        if (!any) return bad;
    }
}

// Parse the first n tokens of the file into out. Returns MVG_OK / MVG_E_IO.
int parse_file(const std::string& path, int64_t n, double* out) {
    int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) return fail(MVG_E_IO, "Unable to open '" + path + "': " + strerror(errno));
    struct stat st;
    if (fstat(fd, &st) != 0) {
        close(fd);
        return fail(MVG_E_IO, "stat failed for '" + path + "'");
    }
    const size_t len = (size_t)st.st_size;
    if (n == 0) {
        close(fd);
        return MVG_OK;
    }
    if (len == 0) {
        close(fd);
        return fail(MVG_E_IO, "'" + path + "' is empty");
    }
    const char* base = (const char*)mmap(nullptr, len, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (base == MAP_FAILED) return fail(MVG_E_IO, "mmap failed for '" + path + "'");

    int nt = host_thread_count();
    if (len < (1u << 20)) nt = 1;
    // nr = nt * kStreams ranges, range r = [cut[r], cut[r+1]), thread t taking ranges
    // [t*kStreams, +kStreams); cuts moved forward to the next whitespace so that no token
    // straddles two ranges.
    const int nr = nt * kStreams;
    std::vector<size_t> cut(nr + 1);
    for (int r = 0; r <= nr; ++r) {
        size_t c = len * (size_t)r / (size_t)nr;
        if (r > 0 && r < nr)
            while (c < len && !is_space(base[c])) ++c;
        cut[r] = c;
    }
    for (int r = 1; r <= nr; ++r)
        if (cut[r] < cut[r - 1]) cut[r] = cut[r - 1];

    std::vector<int64_t> count(nr, 0);
    {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
#ifdef MADV_POPULATE_READ
                // map this thread's pages in one call (page-table batches, no fault per page)
                const size_t lo = cut[t * kStreams] & ~(size_t)4095, hi = cut[(t + 1) * kStreams];
                if (hi > lo) (void)madvise((void*)(base + lo), hi - lo, MADV_POPULATE_READ);
#endif
                for (int r = t * kStreams; r < (t + 1) * kStreams; ++r)
                    count[r] = count_tokens(base + cut[r], base + cut[r + 1]);
            });
        for (auto& x : th) x.join();
    }
    std::vector<int64_t> start(nr + 1, 0);
    for (int r = 0; r < nr; ++r) start[r + 1] = start[r] + count[r];
    if (start[nr] < n) {
        munmap((void*)base, len);
        return fail(MVG_E_IO, "'" + path + "' holds " + std::to_string(start[nr]) +
                                  " values, expected " + std::to_string(n));
    }
    std::vector<int> bad(nt, 0);
    {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                const char* p[kStreams];
                const char* e[kStreams];
                for (int s = 0; s < kStreams; ++s)
                    p[s] = base + cut[t * kStreams + s], e[s] = base + cut[t * kStreams + s + 1];
                bad[t] = parse_ranges(p, e, &start[t * kStreams], n, out);
            });
        for (auto& x : th) x.join();
    }
    munmap((void*)base, len);
    for (int t = 0; t < nt; ++t)
        if (bad[t]) return fail(MVG_E_IO, "'" + path + "' holds a token that is not a number");
    return MVG_OK;
}

// ---- binary cache: "MVGBIN1\0", int64 rows, int64 cols, rows*cols native fp64 (row-major)
constexpr char kMagic[8] = {'M', 'V', 'G', 'B', 'I', 'N', '1', '\0'};
constexpr size_t kHeader = 24;

// Reads the cache into out if it exists, matches (R, C) and is at least as new as the text
// file (when the text exists). Returns MVG_OK, or MVG_E_IO when there is no usable cache.
int read_bin(const std::string& bin, const std::string& txt, int64_t R, int64_t C, double* out) {
    struct stat sb, st;
    if (stat(bin.c_str(), &sb) != 0) return MVG_E_IO;
    if (stat(txt.c_str(), &st) == 0 && st.st_mtime > sb.st_mtime) return MVG_E_IO;  // stale
    const size_t n = (size_t)R * (size_t)C;
    if ((size_t)sb.st_size != kHeader + n * sizeof(double)) return MVG_E_IO;
    int fd = open(bin.c_str(), O_RDONLY);
    if (fd < 0) return MVG_E_IO;
    char hdr[kHeader];
    if (pread(fd, hdr, kHeader, 0) != (ssize_t)kHeader || memcmp(hdr, kMagic, 8) != 0) {
        close(fd);
        return MVG_E_IO;
    }
    int64_t r, c;
    memcpy(&r, hdr + 8, 8);
    memcpy(&c, hdr + 16, 8);
    if (r != R || c != C) {
        close(fd);
        return MVG_E_IO;
    }
    std::vector<int> bad(64, 0);
    const size_t bytes = n * sizeof(double);
    parallel_for((int64_t)((bytes + (64u << 20) - 1) / (64u << 20)), [&](int64_t a, int64_t b) {
        for (int64_t blk = a; blk < b; ++blk) {
            size_t off = (size_t)blk * (64u << 20);
            size_t len = std::min<size_t>(64u << 20, bytes - off);
            char* dst = (char*)out + off;
            while (len > 0) {
                const ssize_t got = pread(fd, dst, len, (off_t)(kHeader + off));
                if (got <= 0) {
                    bad[0] = 1;
                    return;
                }
                dst += got;
                off += (size_t)got;
                len -= (size_t)got;
            }
        }
    }, bytes < (64u << 20));
    close(fd);
    return bad[0] ? MVG_E_IO : MVG_OK;
}

std::string join(const char* dir, const std::string& name) {
    std::string d = dir ? dir : ".";
    if (!d.empty() && d.back() != '/') d += '/';
    return d + name;
}

}  // namespace

extern "C" {

int mvg_matrix_filename(int64_t R, int64_t C, char* buf, size_t buflen) {
    if (!buf) return fail(MVG_E_INVALID, "null");
    int n = snprintf(buf, buflen, "matrix_%lld_%lld.txt", (long long)R, (long long)C);
    return (n < 0 || (size_t)n >= buflen) ? fail(MVG_E_INVALID, "buffer too small") : MVG_OK;
}

int mvg_vector_filename(int64_t n_elems, char* buf, size_t buflen) {
    if (!buf) return fail(MVG_E_INVALID, "null");
    int n = snprintf(buf, buflen, "vector_%lld.txt", (long long)n_elems);
    return (n < 0 || (size_t)n >= buflen) ? fail(MVG_E_INVALID, "buffer too small") : MVG_OK;
}

int mvg_load_matr(const char* dir, int64_t R, int64_t C, double* A) {
    if (R < 0 || C < 0 || (!A && R * C > 0)) return fail(MVG_E_INVALID, "mvg_load_matr: bad arguments");
    char name[128];
    mvg_matrix_filename(R, C, name, sizeof name);
    const std::string txt = join(dir, name);
    std::string bin = txt.substr(0, txt.size() - 4) + ".bin";
    const char* mode = getenv("MVG_BIN_CACHE");  // unset: use a cache if present; "1": also write; "0": off
    const bool use = !(mode && mode[0] == '0');
    if (use && R * C > 0 && read_bin(bin, txt, R, C, A) == MVG_OK) return MVG_OK;
    int rc = parse_file(txt, R * C, A);
    if (rc == MVG_OK && mode && mode[0] == '1') rc = mvg_write_matr_bin(bin.c_str(), A, R, C);
    return rc;
}

int mvg_write_matr_bin(const char* path, const double* A, int64_t R, int64_t C) {
    if (!path || R < 0 || C < 0 || (!A && R * C > 0)) return fail(MVG_E_INVALID, "mvg_write_matr_bin: bad arguments");
    const std::string tmp = std::string(path) + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) return fail(MVG_E_IO, "Unable to create '" + tmp + "'");
    bool ok = fwrite(kMagic, 1, 8, f) == 8 && fwrite(&R, 8, 1, f) == 1 && fwrite(&C, 8, 1, f) == 1;
    const size_t n = (size_t)R * (size_t)C;
    for (size_t off = 0; ok && off < n; off += (size_t)1 << 24) {
        const size_t len = std::min<size_t>((size_t)1 << 24, n - off);
        ok = fwrite(A + off, sizeof(double), len, f) == len;
    }
    ok = (fclose(f) == 0) && ok;
    if (!ok || rename(tmp.c_str(), path) != 0) {
        remove(tmp.c_str());
        return fail(MVG_E_IO, std::string("write failed for '") + path + "'");
    }
    return MVG_OK;
}

int mvg_load_vec(const char* dir, int64_t n, double* x) {
    if (n < 0 || (!x && n > 0)) return fail(MVG_E_INVALID, "mvg_load_vec: bad arguments");
    char name[128];
    mvg_vector_filename(n, name, sizeof name);
    return parse_file(join(dir, name), n, x);
}

int mvg_write_vec(const char* path, const double* v, int64_t n) {
    if (!path || n < 0 || (!v && n > 0)) return fail(MVG_E_INVALID, "mvg_write_vec: bad arguments");
    FILE* f = fopen(path, "w");
    if (!f) return fail(MVG_E_IO, std::string("Unable to create '") + path + "'");
    for (int64_t i = 0; i < n; ++i) fprintf(f, "%.17g\n", v[i]);
    if (fclose(f) != 0) return fail(MVG_E_IO, std::string("write failed for '") + path + "'");
    return MVG_OK;
}

// "%.4f " per value, one matrix row per line (the reference's numpy-written format,
// README.md:32). Rows are formatted in parallel into per-thread buffers, written in order.
int mvg_write_matr_synth(const char* path, int64_t R, int64_t C, uint64_t seed) {
    if (!path || R < 0 || C < 0) return fail(MVG_E_INVALID, "mvg_write_matr_synth: bad arguments");
    FILE* f = fopen(path, "w");
    if (!f) return fail(MVG_E_IO, std::string("Unable to create '") + path + "'");
    const uint64_t s0 = splitmix64(seed);
    const int64_t rows_per_batch = C > 0 ? std::max<int64_t>(1, (64ll << 20) / (C * 8)) : R;
    for (int64_t r0 = 0; r0 < R; r0 += rows_per_batch) {
        const int64_t r1 = std::min(R, r0 + rows_per_batch);
        std::vector<std::string> lines(r1 - r0);
        parallel_for(r1 - r0, [&](int64_t a, int64_t b) {
            char tmp[32];
            for (int64_t r = a; r < b; ++r) {
                std::string& s = lines[r];
                s.reserve((size_t)C * 7 + 1);
                const uint64_t gbase = (uint64_t)(r0 + r) * (uint64_t)C;
                for (int64_t c = 0; c < C; ++c) {
                    int l = snprintf(tmp, sizeof tmp, "%.4f ", synth_value(s0, gbase + c));
                    s.append(tmp, (size_t)l);
                }
                s.push_back('\n');
            }
        }, (r1 - r0) * C < (1 << 16));
        for (auto& s : lines) fwrite(s.data(), 1, s.size(), f);
    }
    if (fclose(f) != 0) return fail(MVG_E_IO, std::string("write failed for '") + path + "'");
    return MVG_OK;
}

}  // extern "C"
