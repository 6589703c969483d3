// mhs_mmio.cpp -- Matrix Market -> CSR reader and host helpers of the C-ABI.
//
// Semantics follow readMtxFile (reference inc/mmio_read.h:34-159) and the banner
// / size parsers (inc/mmio.h:128-232):
//   * banner "%%MatrixMarket matrix coordinate <real|integer|pattern|complex>
//     <general|symmetric|hermitian|skew-symmetric>", tokens case-insensitive;
//   * '%' comment lines skipped before "M N nnz";
//   * values: real as double, integer converted to double, pattern = 1.0,
//     complex keeps the real part;
//   * 1-based -> 0-based; symmetric and hermitian off-diagonal entries are
//     mirrored with the same value; skew-symmetric entries are NOT mirrored
//     (the reference only tests is_symmetric || is_hermitian, :112);
//   * CSR filled in file order (entry, then its mirror), duplicates kept,
//     each row sorted by (col, val) pairs (:9-31, :150).
// Unlike the reference (one fscanf per token), the file is read in one block
// and tokenised in parallel chunks; rows are sorted in parallel.
#include "../../include/mhspgemm.h"

#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace {

int hw_threads() {
    unsigned n = std::thread::hardware_concurrency();
    if (n == 0) n = 1;
    if (n > 32) n = 32;
    return (int)n;
}

template <class F>
void parallel_for(long long n, F f) {
    const int T = hw_threads();
    if (n < 4096 || T == 1) {
        f(0LL, n, 0);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) {
        const long long lo = n * t / T, hi = n * (t + 1) / T;
        th.emplace_back([=] { f(lo, hi, t); });
    }
    for (auto& x : th) x.join();
}

bool read_line(const char*& p, const char* end, std::string& line) {
    if (p >= end) return false;
    const char* q = (const char*)memchr(p, '\n', (size_t)(end - p));
    if (!q) q = end;
    line.assign(p, q);
    p = q < end ? q + 1 : end;
    return true;
}

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; }

struct Entry {
    int r, c;
    double v;
};

constexpr char kBinMagic[8] = {'M', 'H', 'S', 'C', 'S', 'R', '\0', '\0'};
constexpr int32_t kBinVersion = 1;

struct BinHeader {
    char magic[8];
    int32_t version, M, N, nnz, is_symmetric, pad0;
    int64_t src_size, src_mtime_ns;
    int64_t pad1[2];
};
static_assert(sizeof(BinHeader) == 64, "binary CSR header is 64 bytes");

}  // namespace

extern "C" {

void mhs_host_csr_free(mhs_host_csr* A) {
    if (!A) return;
    free(A->ptr);
    free(A->col);
    free(A->val);
    std::memset(A, 0, sizeof *A);
}

uint64_t mhs_flop_count(int32_t nnzA, const int32_t* Acol, const int32_t* Bptr) {
    uint64_t s = 0;
    for (int32_t j = 0; j < nnzA; ++j) s += (uint64_t)(Bptr[Acol[j] + 1] - Bptr[Acol[j]]);
    return s;
}

int mhs_read_mtx(const char* path, mhs_host_csr* A) {
    if (!A) return MHS_ERR_INVALID;
    std::memset(A, 0, sizeof *A);
    FILE* f = fopen(path, "rb");
    if (!f) return MHS_ERR_IO;
    std::vector<char> buf;
    {
        if (fseek(f, 0, SEEK_END) != 0) {
            fclose(f);
            return MHS_ERR_IO;
        }
        const long sz = ftell(f);
        if (sz < 0) {
            fclose(f);
            return MHS_ERR_IO;
        }
        fseek(f, 0, SEEK_SET);
        buf.resize((size_t)sz + 1);
        const size_t got = fread(buf.data(), 1, (size_t)sz, f);
        fclose(f);
        if (got != (size_t)sz) return MHS_ERR_IO;
        buf[(size_t)sz] = '\0';
    }
    const char* p = buf.data();
    const char* end = p + buf.size() - 1;
    std::string line;
    // banner
    if (!read_line(p, end, line)) return MHS_ERR_IO;
    char tok[5][64];
    if (sscanf(line.c_str(), "%63s %63s %63s %63s %63s", tok[0], tok[1], tok[2], tok[3], tok[4]) != 5)
        return MHS_ERR_IO;
    for (int i = 1; i < 5; ++i)
        for (char* c = tok[i]; *c; ++c) *c = (char)tolower((unsigned char)*c);
    if (strncmp(tok[0], "%%MatrixMarket", 14) != 0 || strcmp(tok[1], "matrix") != 0) return MHS_ERR_IO;
    if (strcmp(tok[2], "coordinate") != 0) return MHS_ERR_IO;  // dense "array" storage unsupported
    char type;
    if (!strcmp(tok[3], "real")) type = 'R';
    else if (!strcmp(tok[3], "integer")) type = 'I';
    else if (!strcmp(tok[3], "pattern")) type = 'P';
    else if (!strcmp(tok[3], "complex")) type = 'C';
    else return MHS_ERR_IO;
    char storage;
    if (!strcmp(tok[4], "general")) storage = 'G';
    else if (!strcmp(tok[4], "symmetric")) storage = 'S';
    else if (!strcmp(tok[4], "hermitian")) storage = 'H';
    else if (!strcmp(tok[4], "skew-symmetric")) storage = 'K';
    else return MHS_ERR_IO;
    // size line
    int M = 0, N = 0, nz = 0;
    for (;;) {
        if (!read_line(p, end, line)) return MHS_ERR_IO;
        if (!line.empty() && line[0] == '%') continue;
        if (sscanf(line.c_str(), "%d %d %d", &M, &N, &nz) == 3) break;
        // blank line: keep scanning tokens (mm_read_mtx_crd_size's fscanf loop)
        bool blank = true;
        for (char c : line) blank &= is_space(c);
        if (!blank) return MHS_ERR_IO;
    }
    if (M < 0 || N < 0 || nz < 0) return MHS_ERR_IO;
    const int per = type == 'P' ? 2 : type == 'C' ? 4 : 3;  // tokens per entry
    // Tokenise the body in parallel: chunk boundaries snapped to line ends,
    // each chunk counts its tokens, then parses into its slot range.
    const long long body = end - p;
    const int T = body > (1 << 20) ? hw_threads() : 1;
    std::vector<const char*> cs(T + 1);
    cs[0] = p;
    cs[T] = end;
    for (int t = 1; t < T; ++t) {
        const char* q = p + body * t / T;
        if (q < cs[t - 1]) q = cs[t - 1];
        while (q < end && *q != '\n') ++q;
        cs[t] = q < end ? q + 1 : end;
    }
    std::vector<long long> ntok(T + 1, 0);
    auto count_tokens = [&](int t) {
        long long n = 0;
        const char* q = cs[t];
        const char* e = cs[t + 1];
        bool in = false;
        for (; q < e; ++q) {
            const bool sp = is_space(*q);
            if (!sp && !in) ++n;
            in = !sp;
        }
        ntok[t + 1] = n;
    };
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) th.emplace_back(count_tokens, t);
        for (auto& x : th) x.join();
    }
    for (int t = 0; t < T; ++t) ntok[t + 1] += ntok[t];
    if (ntok[T] < (long long)nz * per) return MHS_ERR_IO;
    std::vector<Entry> ent((size_t)nz);
    std::vector<int> bad(T, 0);
    auto parse = [&](int t) {
        long long k = ntok[t];  // global token index of this chunk's first token
        const long long kmax = (long long)nz * per;
        const char* q = cs[t];
        const char* e = cs[t + 1];
        while (q < e && k < kmax) {
            while (q < e && is_space(*q)) ++q;
            if (q >= e) break;
            const long long idx = k / per;
            const int fld = (int)(k % per);
            char* nx = nullptr;
            Entry& x = ent[(size_t)idx];
            if (fld == 0 || fld == 1) {
                const long v = strtol(q, &nx, 10);
                if (nx == q) {
                    bad[t] = 1;
                    return;
                }
                if (fld == 0) x.r = (int)v - 1;
                else x.c = (int)v - 1;
                if (type == 'P' && fld == 1) x.v = 1.0;
            } else if (fld == 2) {
                if (type == 'I') {
                    const long v = strtol(q, &nx, 10);
                    x.v = (double)(int)v;
                } else {
                    x.v = strtod(q, &nx);
                }
                if (nx == q) {
                    bad[t] = 1;
                    return;
                }
            } else {  // imaginary part: parsed and dropped
                (void)strtod(q, &nx);
                if (nx == q) {
                    bad[t] = 1;
                    return;
                }
            }
            q = nx;
            ++k;
        }
    };
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) th.emplace_back(parse, t);
        for (auto& x : th) x.join();
    }
    for (int t = 0; t < T; ++t)
        if (bad[t]) return MHS_ERR_IO;
    const bool sym = storage == 'S' || storage == 'H';
    std::vector<int64_t> cnt((size_t)M + 1, 0);
    for (const Entry& x : ent) {
        if (x.r < 0 || x.r >= M || x.c < 0 || x.c >= N) return MHS_ERR_IO;
        cnt[(size_t)x.r]++;
        if (sym && x.r != x.c) {
            if (x.c >= M) return MHS_ERR_IO;
            cnt[(size_t)x.c]++;
        }
    }
    int64_t run = 0;
    for (int r = 0; r <= M; ++r) {
        const int64_t c = cnt[(size_t)r];
        cnt[(size_t)r] = run;
        run += c;
    }
    if (run > 0x7fffffff) return MHS_ERR_IO;
    A->M = M;
    A->N = N;
    A->nnz = (int32_t)run;
    A->is_symmetric = storage == 'S';
    A->ptr = (int32_t*)malloc(sizeof(int32_t) * ((size_t)M + 1));
    A->col = (int32_t*)malloc(sizeof(int32_t) * (size_t)(run > 0 ? run : 1));
    A->val = (double*)malloc(sizeof(double) * (size_t)(run > 0 ? run : 1));
    if (!A->ptr || !A->col || !A->val) {
        mhs_host_csr_free(A);
        return MHS_ERR_IO;
    }
    for (int r = 0; r <= M; ++r) A->ptr[r] = (int32_t)cnt[(size_t)r];
    std::vector<int32_t> fill((size_t)M + 1, 0);
    for (const Entry& x : ent) {
        int32_t o = A->ptr[x.r] + fill[(size_t)x.r]++;
        A->col[o] = x.c;
        A->val[o] = x.v;
        if (sym && x.r != x.c) {
            o = A->ptr[x.c] + fill[(size_t)x.c]++;
            A->col[o] = x.r;
            A->val[o] = x.v;
        }
    }
    parallel_for(M, [&](long long lo, long long hi, int) {
        std::vector<std::pair<int32_t, double>> row;
        for (long long r = lo; r < hi; ++r) {
            const int32_t s = A->ptr[r], e = A->ptr[r + 1];
            if (e - s < 2) continue;
            bool sorted = true;
            for (int32_t j = s + 1; j < e && sorted; ++j)
                sorted = A->col[j - 1] < A->col[j] ||
                         (A->col[j - 1] == A->col[j] && A->val[j - 1] <= A->val[j]);
            if (sorted) continue;
            row.clear();
            for (int32_t j = s; j < e; ++j) row.emplace_back(A->col[j], A->val[j]);
            std::sort(row.begin(), row.end());
            for (int32_t j = s; j < e; ++j) {
                A->col[j] = row[(size_t)(j - s)].first;
                A->val[j] = row[(size_t)(j - s)].second;
            }
        }
    });
    return MHS_OK;
}

// ---- binary CSR cache (the text parse of cage15 / wb-edu / GAP-road is
// the step before the path; inc/mmio_read.h:80-108 re-parses with fscanf on every run).
// File: a 64-byte header {magic, version, M, N, nnz, is_symmetric, source size, source
// mtime (ns)}, then ptr[M+1] int32, col[nnz] int32, val[nnz] f64, little-endian as on the
// host.  The source's size + mtime stamp the cache: a rewritten .mtx invalidates it.

int mhs_write_csr_bin(const char* path, const mhs_host_csr* A, int64_t src_size, int64_t src_mtime_ns) {
    if (!path || !A || A->M < 0 || A->nnz < 0 || !A->ptr || (A->nnz > 0 && (!A->col || !A->val)))
        return MHS_ERR_INVALID;
    BinHeader h{};
    std::memcpy(h.magic, kBinMagic, sizeof h.magic);
    h.version = kBinVersion;
    h.M = A->M;
    h.N = A->N;
    h.nnz = A->nnz;
    h.is_symmetric = A->is_symmetric;
    h.src_size = src_size;
    h.src_mtime_ns = src_mtime_ns;
    // write to a temporary name and rename: a reader never sees a half-written cache
    const std::string tmp = std::string(path) + ".tmp" + std::to_string((long long)getpid());
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) return MHS_ERR_IO;
    bool ok = fwrite(&h, sizeof h, 1, f) == 1 &&
              fwrite(A->ptr, sizeof(int32_t), (size_t)A->M + 1, f) == (size_t)A->M + 1 &&
              (A->nnz == 0 || (fwrite(A->col, sizeof(int32_t), (size_t)A->nnz, f) == (size_t)A->nnz &&
                               fwrite(A->val, sizeof(double), (size_t)A->nnz, f) == (size_t)A->nnz));
    ok = (fclose(f) == 0) && ok;
    if (!ok || rename(tmp.c_str(), path) != 0) {
        unlink(tmp.c_str());
        return MHS_ERR_IO;
    }
    return MHS_OK;
}

int mhs_read_csr_bin(const char* path, mhs_host_csr* A, int64_t* src_size, int64_t* src_mtime_ns) {
    if (!A) return MHS_ERR_INVALID;
    std::memset(A, 0, sizeof *A);
    FILE* f = fopen(path, "rb");
    if (!f) return MHS_ERR_IO;
    BinHeader h{};
    if (fread(&h, sizeof h, 1, f) != 1 || std::memcmp(h.magic, kBinMagic, sizeof h.magic) != 0 ||
        h.version != kBinVersion || h.M < 0 || h.N < 0 || h.nnz < 0) {
        fclose(f);
        return MHS_ERR_IO;
    }
    const size_t nz = (size_t)h.nnz;
    A->ptr = (int32_t*)malloc(sizeof(int32_t) * ((size_t)h.M + 1));
    A->col = (int32_t*)malloc(sizeof(int32_t) * (nz > 0 ? nz : 1));
    A->val = (double*)malloc(sizeof(double) * (nz > 0 ? nz : 1));
    bool ok = A->ptr && A->col && A->val &&
              fread(A->ptr, sizeof(int32_t), (size_t)h.M + 1, f) == (size_t)h.M + 1 &&
              (nz == 0 || (fread(A->col, sizeof(int32_t), nz, f) == nz &&
                           fread(A->val, sizeof(double), nz, f) == nz));
    fclose(f);
    // a truncated or corrupt cache must not reach the device: check the CSR invariants
    ok = ok && A->ptr[0] == 0 && A->ptr[h.M] == h.nnz;
    if (ok) {
        std::atomic<bool> good{true};
        parallel_for(h.M, [&](long long lo, long long hi, int) {
            for (long long r = lo; r < hi && good.load(std::memory_order_relaxed); ++r) {
                const int32_t s = A->ptr[r], e = A->ptr[r + 1];
                if (e < s || e > h.nnz) {
                    good = false;
                    return;
                }
                for (int32_t j = s; j < e; ++j)
                    if ((uint32_t)A->col[j] >= (uint32_t)h.N) {
                        good = false;
                        return;
                    }
            }
        });
        ok = good.load();
    }
    if (!ok) {
        mhs_host_csr_free(A);
        return MHS_ERR_IO;
    }
    A->M = h.M;
    A->N = h.N;
    A->nnz = h.nnz;
    A->is_symmetric = h.is_symmetric;
    if (src_size) *src_size = h.src_size;
    if (src_mtime_ns) *src_mtime_ns = h.src_mtime_ns;
    return MHS_OK;
}

int mhs_read_mtx_cached(const char* path, const char* cache_path, mhs_host_csr* A, int* from_cache) {
    if (!path || !A) return MHS_ERR_INVALID;
    if (from_cache) *from_cache = 0;
    struct stat st;
    if (stat(path, &st) != 0) return MHS_ERR_IO;
    const int64_t size = (int64_t)st.st_size;
    const int64_t mtime = (int64_t)st.st_mtim.tv_sec * 1000000000LL + (int64_t)st.st_mtim.tv_nsec;
    const std::string cache = cache_path && *cache_path ? std::string(cache_path) : std::string(path) + ".mhscsr";
    int64_t cs = -1, cm = -1;
    if (mhs_read_csr_bin(cache.c_str(), A, &cs, &cm) == MHS_OK) {
        if (cs == size && cm == mtime) {
            if (from_cache) *from_cache = 1;
            return MHS_OK;
        }
        mhs_host_csr_free(A);  // stale: the .mtx changed since the cache was written
    }
    const int rc = mhs_read_mtx(path, A);
    if (rc != MHS_OK) return rc;
    (void)mhs_write_csr_bin(cache.c_str(), A, size, mtime);  // best effort (read-only dirs)
    return MHS_OK;
}

}  // extern "C"
