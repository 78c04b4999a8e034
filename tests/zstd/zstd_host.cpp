// Serial zstd encoder over the device encoder's building blocks
// (acquire-zarr_amd/csrc/aqz_zstd.hh), decoded by libzstd.
//
// It is the CPU check of every format piece the GPU kernels emit (frame and
// block headers, Huffman tree description with FSE-compressed or direct
// weights, 4-stream Huffman literals, Treeless literals, RLE blocks,
// predefined-FSE sequences) and, for literal-only frames, the byte-exact
// model of the device encoder's output (tests/test_gpu_zstd.py compares
// the two through libzstd_host.so).  Usage: zstd_host LIBZSTD_PATH
#include "aqz_zstd.hh"

#include <dlfcn.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

using namespace aqz::zstd;

namespace {

struct Table
{
    int mode = 0; // 0 raw literals, 1 one symbol, 2 Huffman
    uint8_t len[256];
    uint16_t code[256];
    uint8_t tree[160];
    uint32_t tree_n = 0;
};

Table
make_table(const uint32_t* hist)
{
    Table t;
    uint32_t present = 0, mx = 0;
    uint64_t total = 0;
    for (int k = 0; k < 256; ++k) {
        present += hist[k] != 0;
        mx = hist[k] > mx ? hist[k] : mx;
        total += hist[k];
    }
    if (huf_flat(present, mx, total)) {
        std::memset(t.len, 0, sizeof t.len);
        return t; // raw literals
    }
    const uint32_t n = huf_lengths(hist, t.len, kHufMaxBits);
    if (n == 1)
        t.mode = 1;
    if (n >= 2) {
        const uint32_t mb = huf_codes(t.len, t.code);
        t.tree_n = huf_write_tree(t.len, mb, t.tree);
        t.mode = t.tree_n ? 2 : 0;
    }
    return t;
}

// 4 Huffman streams of lit[0..n) -> out (jump table + streams); bytes
uint32_t
huf_streams(const Table& t, const uint8_t* lit, uint32_t n, uint8_t* out, uint32_t cap)
{
    const uint32_t seg = lit_segment(n);
    uint32_t at = 6, sz[4];
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t a = std::min(n, k * seg), b = std::min(n, (k + 1) * seg);
        // the device keeps a stream only when it fits 8 bits per literal
        // (+ 32): the same rule here
        uint64_t bits = 0;
        for (uint32_t i = a; i < b; ++i)
            bits += t.len[lit[i]];
        if (bits + 1 > 8ull * (b - a) + 32)
            return 0;
        BitW w;
        w.init(out + at, cap > at ? cap - at : 0);
        for (uint32_t i = b; i-- > a;)
            w.add(t.code[lit[i]], t.len[lit[i]]);
        sz[k] = w.close();
        if (sz[k] == 0 || sz[k] > 65535)
            return 0;
        at += sz[k];
    }
    put_le(out, sz[0], 2);
    put_le(out + 2, sz[1], 2);
    put_le(out + 4, sz[2], 2);
    return at;
}

constexpr uint32_t kMinHuf = 64; // fewer literals: stored raw
constexpr uint32_t kGroupLog2 = 3; // blocks per Huffman table: 8 (the device's kHufGroup)

// how often each format path was taken (the run must take every one)
struct Paths
{
    uint64_t rle_block, raw_block, cmp_block, tree_fse, tree_direct, treeless, rle_lit,
      raw_lit, seqs;
} g_paths{};

// greedy LZ parse of one block (hash of 4 bytes, min match 4)
void
parse(const uint8_t* b, uint32_t n, std::vector<Seq>& seqs, std::vector<uint8_t>& lits)
{
    seqs.clear();
    lits.clear();
    std::vector<int32_t> table(1 << 14, -1);
    auto rd = [&](uint32_t p) {
        uint32_t v;
        std::memcpy(&v, b + p, 4);
        return v;
    };
    // a match pays when its length times the literal cost (~ the block's
    // byte entropy) beats a sequence's ~MATCH_BITS bits
    uint32_t h256[256] = { 0 };
    for (uint32_t i = 0; i < n; ++i)
        h256[b[i]]++;
    double H = 0;
    for (uint32_t k = 0; k < 256; ++k)
        if (h256[k])
            H -= double(h256[k]) / n * std::log2(double(h256[k]) / n);
    const char* mb = std::getenv("MATCH_BITS");
    uint32_t minlen = min_match(float(H), 64);
    if (mb) // sweep hook: bits a match must save (0: every 4-byte match)
        minlen = std::atof(mb) > 0
                   ? uint32_t(std::min(64.0, std::max(4.0, std::ceil(std::atof(mb) / std::max(H, 0.25)))))
                   : 4;
    uint32_t anchor = 0, p = 0;
    while (p + 4 <= n) {
        const uint32_t v = rd(p);
        const uint32_t h = (v * 2654435761u) >> 18;
        const int32_t c = table[h];
        table[h] = int32_t(p);
        if (c >= 0 && rd(uint32_t(c)) == v) {
            uint32_t len = 4;
            while (p + len < n && b[c + len] == b[p + len])
                ++len;
            if (len < minlen) {
                ++p;
                continue;
            }
            seqs.push_back(Seq{ p - anchor, len, p - uint32_t(c) });
            lits.insert(lits.end(), b + anchor, b + p);
            for (uint32_t q = p + 1; q < p + len && q + 4 <= n; q += 3)
                table[(rd(q) * 2654435761u) >> 18] = int32_t(q);
            p += len;
            anchor = p;
        } else {
            ++p;
        }
    }
    lits.insert(lits.end(), b + anchor, b + n);
}

// One frame of src[0..n); lz = with sequences.  The decision rule matches
// the device encoder: a block is compressed iff its content, counted with
// the tree description, is smaller than the block.
std::vector<uint8_t>
encode_frame(const uint8_t* src, uint64_t n, bool lz, const SeqTables& st,
             uint32_t glog2 = kGroupLog2)
{
    std::vector<uint8_t> out(frame_header_bytes(n) + n + 3 * (n / kBlock + 1) + 64);
    uint32_t at = write_frame_header(out.data(), n);
    const uint32_t nb = uint32_t((n + kBlock - 1) / kBlock);
    // parse every block; the literal histogram of each group of 2^glog2
    // blocks (the device's Huffman groups, aqz_codec.hh zstd_huf_group_log2)
    std::vector<std::vector<Seq>> bseq(nb);
    std::vector<std::vector<uint8_t>> blit(nb);
    const uint32_t ng = (nb + (1u << glog2) - 1) >> glog2;
    std::vector<std::vector<uint32_t>> ghist(ng, std::vector<uint32_t>(256, 0));
    for (uint32_t j = 0; j < nb; ++j) {
        const uint8_t* b = src + uint64_t(j) * kBlock;
        const uint32_t bn = uint32_t(std::min<uint64_t>(kBlock, n - uint64_t(j) * kBlock));
        if (lz)
            parse(b, bn, bseq[j], blit[j]);
        else
            blit[j].assign(b, b + bn);
        for (uint8_t x : blit[j])
            ghist[j >> glog2][x]++;
    }
    std::vector<Table> gt(ng);
    for (uint32_t k = 0; k < ng; ++k)
        gt[k] = make_table(ghist[k].data());
    std::vector<bool> gsent(ng, false);
    std::vector<uint8_t> tmp(2 * kBlock + 1024);
    for (uint32_t j = 0; j < nb; ++j) {
        const uint8_t* b = src + uint64_t(j) * kBlock;
        const uint32_t bn = uint32_t(std::min<uint64_t>(kBlock, n - uint64_t(j) * kBlock));
        const bool last = j + 1 == nb;
        bool same = true;
        for (uint32_t i = 1; i < bn && same; ++i)
            same = b[i] == b[0];
        if (same) {
            g_paths.rle_block++;
            write_block_header(out.data() + at, last, 1, bn);
            out[at + 3] = b[0];
            at += 4;
            continue;
        }
        const std::vector<uint8_t>& L = blit[j];
        const uint32_t nl = uint32_t(L.size());
        const Table& t = gt[j >> glog2];
        const bool tree_sent = gsent[j >> glog2];
        // literals section into tmp
        uint32_t lsz = 0, tree_extra = 0; // tree bytes a later block would not carry
        bool used_tree = false;
        bool lsame = nl > 0;
        for (uint32_t i = 1; i < nl && lsame; ++i)
            lsame = L[i] == L[0];
        if (lsame && nl >= 2) {
            lsz = write_lit_header_raw(tmp.data(), 1, nl);
            tmp[lsz++] = L[0];
        } else if (t.mode == 2 && nl >= kMinHuf) {
            std::vector<uint8_t> s(nl + nl / 2 + 64);
            const uint32_t sn = huf_streams(t, L.data(), nl, s.data(), uint32_t(s.size()));
            const uint32_t with_tree = t.tree_n + sn;
            // raw literals unless Huffman (counted with the tree) is smaller
            if (sn && with_tree + lit_header_huf_bytes(nl, with_tree) < nl + lit_header_raw_bytes(nl)) {
                const uint32_t cs = (tree_sent ? 0 : t.tree_n) + sn;
                lsz = write_lit_header_huf(tmp.data(), tree_sent ? 3 : 2, nl, cs);
                if (tree_sent) // decide as if the tree were carried
                    tree_extra = t.tree_n + lit_header_huf_bytes(nl, with_tree) -
                                 lit_header_huf_bytes(nl, cs);
                if (!tree_sent) {
                    std::memcpy(tmp.data() + lsz, t.tree, t.tree_n);
                    lsz += t.tree_n;
                    used_tree = true;
                }
                std::memcpy(tmp.data() + lsz, s.data(), sn);
                lsz += sn;
            }
        }
        if (lsz == 0) {
            lsz = write_lit_header_raw(tmp.data(), 0, nl);
            std::memcpy(tmp.data() + lsz, L.data(), nl);
            lsz += nl;
        }
        uint32_t csz = lsz + write_seq_header(tmp.data() + lsz, uint32_t(bseq[j].size()));
        if (!bseq[j].empty()) {
            const std::vector<Seq>& sv = bseq[j];
            const uint32_t q = encode_sequences(
              st, [&](uint32_t i) { return sv[i]; }, uint32_t(sv.size()), tmp.data() + csz,
              uint32_t(tmp.size()) - csz);
            if (q == 0) {
                std::fprintf(stderr, "sequence stream overflow\n");
                std::exit(3);
            }
            csz += q;
        }
        if (csz + tree_extra >= bn) { // raw block
            g_paths.raw_block++;
            write_block_header(out.data() + at, last, 0, bn);
            std::memcpy(out.data() + at + 3, b, bn);
            at += 3 + bn;
            continue;
        }
        if (used_tree)
            gsent[j >> glog2] = true;
        g_paths.cmp_block++;
        if (used_tree)
            (t.tree[0] < 128 ? g_paths.tree_fse : g_paths.tree_direct)++;
        else if (tmp[0] % 4 == 3)
            g_paths.treeless++;
        else if (tmp[0] % 4 == 1)
            g_paths.rle_lit++;
        else
            g_paths.raw_lit++;
        if (!bseq[j].empty())
            g_paths.seqs++;
        write_block_header(out.data() + at, last, 2, csz);
        std::memcpy(out.data() + at + 3, tmp.data(), csz);
        at += 3 + csz;
    }
    if (nb == 0) { // empty content: one empty raw block
        write_block_header(out.data() + at, true, 0, 0);
        at += 3;
    }
    out.resize(at);
    return out;
}

} // namespace

// ctypes entry (tests/test_gpu_zstd.py): the frame of src[0..n) into out;
// bytes, 0 when cap is too small.
extern "C" uint64_t
zh_encode_frame_g(const uint8_t* src, uint64_t n, int lz, uint32_t glog2, uint8_t* out,
                  uint64_t cap)
{
    static SeqTables st;
    static const bool ok = build_seq_tables(st);
    if (!ok || glog2 > 5)
        return 0;
    const std::vector<uint8_t> f = encode_frame(src, n, lz != 0, st, glog2);
    if (f.size() > cap)
        return 0;
    std::memcpy(out, f.data(), f.size());
    return f.size();
}

// the same with the default group of 8 blocks
extern "C" uint64_t
zh_encode_frame(const uint8_t* src, uint64_t n, int lz, uint8_t* out, uint64_t cap)
{
    return zh_encode_frame_g(src, n, lz, kGroupLog2, out, cap);
}

namespace {

using dec_t = size_t (*)(void*, size_t, const void*, size_t);
using err_t = unsigned (*)(size_t);
using name_t = const char* (*)(size_t);
using cmp_t = size_t (*)(void*, size_t, const void*, size_t, int);

std::vector<uint8_t>
payload(const std::string& kind, uint64_t n, std::mt19937& rng)
{
    std::vector<uint8_t> v(n);
    std::normal_distribution<double> nd(0.0, 30.0);
    if (kind == "zeros")
        return v;
    if (kind == "random") {
        for (auto& x : v)
            x = uint8_t(rng());
    } else if (kind == "camera16" || kind == "camera16_shuf") {
        const uint64_t np = n / 2;
        std::vector<uint16_t> px(np);
        for (uint64_t i = 0; i < np; ++i)
            px[i] = uint16_t(std::max(0.0, 1000 + 200 * std::sin(double(i) / 977.0) + nd(rng)));
        if (kind == "camera16") {
            std::memcpy(v.data(), px.data(), 2 * np);
        } else { // byte shuffle in 256 KiB blocks
            for (uint64_t b0 = 0; b0 < np; b0 += 131072) {
                const uint64_t m = std::min<uint64_t>(131072, np - b0);
                for (uint64_t i = 0; i < m; ++i) {
                    v[2 * b0 + i] = uint8_t(px[b0 + i]);
                    v[2 * b0 + m + i] = uint8_t(px[b0 + i] >> 8);
                }
            }
        }
    } else if (kind == "sparse") {
        for (uint64_t i = 0; i < n; i += 1 + rng() % 300)
            v[i] = uint8_t(rng());
    } else if (kind == "skewed") { // a few symbols, very unequal
        for (auto& x : v) {
            const uint32_t r = rng() % 1000;
            x = r < 900 ? 7 : r < 990 ? 9 : uint8_t(rng() % 40);
        }
    } else if (kind == "wide") { // > 128 symbols, peaked: FSE weights
        for (auto& x : v)
            x = uint8_t(128 + int(nd(rng) / 3));
    } else if (kind == "binary") { // two symbols: a 1-weight direct tree
        for (auto& x : v)
            x = uint8_t(rng() % 5 == 0);
    } else if (kind == "text") {
        const char* w[] = { "zarr ", "chunk ", "shard ", "level ", "frame ", "the ", "of " };
        uint64_t i = 0;
        while (i < n) {
            const char* s = w[rng() % 7];
            for (const char* c = s; *c && i < n; ++c)
                v[i++] = uint8_t(*c);
        }
    }
    return v;
}

} // namespace

int
main(int argc, char** argv)
{
    const char* libp = argc > 1 ? argv[1] : "libzstd.so.1";
    void* h = dlopen(libp, RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        std::fprintf(stderr, "cannot load %s\n", libp);
        return 2;
    }
    auto dec = reinterpret_cast<dec_t>(dlsym(h, "ZSTD_decompress"));
    auto iserr = reinterpret_cast<err_t>(dlsym(h, "ZSTD_isError"));
    auto ename = reinterpret_cast<name_t>(dlsym(h, "ZSTD_getErrorName"));
    auto cmp = reinterpret_cast<cmp_t>(dlsym(h, "ZSTD_compress"));
    SeqTables st;
    if (!build_seq_tables(st)) {
        std::fprintf(stderr, "predefined tables invalid\n");
        return 2;
    }
    std::mt19937 rng(5);
    const char* kinds[] = { "zeros", "random", "camera16", "camera16_shuf", "sparse",
                            "skewed", "wide", "text", "binary" };
    const uint64_t sizes[] = { 0, 1, 5, 63, 64, 100, 1000, 4096, 32767, 32768, 32769,
                               100000, 262144, 1 << 20 };
    uint64_t frames = 0;
    for (const char* k : kinds) {
        uint64_t in_b = 0, out_b[2] = { 0, 0 }, ref_b[2] = { 0, 0 };
        for (uint64_t n : sizes)
            for (int lz = 0; lz < 2; ++lz) {
                const std::vector<uint8_t> src = payload(k, n, rng);
                const std::vector<uint8_t> f = encode_frame(src.data(), n, lz != 0, st);
                std::vector<uint8_t> back(n + 1);
                const size_t r = dec(back.data(), back.size(), f.data(), f.size());
                if (iserr(r) || r != n || std::memcmp(back.data(), src.data(), n) != 0) {
                    std::fprintf(stderr, "FAIL kind=%s n=%llu lz=%d: %s (got %zu)\n", k,
                                 (unsigned long long)n, lz, iserr(r) ? ename(r) : "mismatch",
                                 iserr(r) ? size_t(0) : r);
                    return 1;
                }
                ++frames;
                if (n >= 262144) {
                    in_b += lz ? 0 : n;
                    out_b[lz] += f.size();
                    std::vector<uint8_t> z(n + n / 128 + 1024);
                    const size_t zn = cmp(z.data(), z.size(), src.data(), n, lz ? 3 : 1);
                    ref_b[lz] += iserr(zn) ? n : zn;
                }
            }
        std::printf("  %-14s ratio: literals only %7.3f, with matches %7.3f | libzstd level 1 "
                    "%7.3f, level 3 %7.3f\n",
                    k, double(in_b) / double(out_b[0]), double(in_b) / double(out_b[1]),
                    double(in_b) / double(ref_b[0]), double(in_b) / double(ref_b[1]));
    }
    const Paths& q = g_paths;
    std::printf("paths: rle_block %llu raw_block %llu compressed %llu (tree fse %llu, tree "
                "direct %llu, treeless %llu, rle literals %llu, raw literals %llu, with "
                "sequences %llu)\n",
                (unsigned long long)q.rle_block, (unsigned long long)q.raw_block,
                (unsigned long long)q.cmp_block, (unsigned long long)q.tree_fse,
                (unsigned long long)q.tree_direct, (unsigned long long)q.treeless,
                (unsigned long long)q.rle_lit, (unsigned long long)q.raw_lit,
                (unsigned long long)q.seqs);
    if (!q.rle_block || !q.raw_block || !q.tree_fse || !q.tree_direct || !q.treeless ||
        !q.raw_lit || !q.seqs) {
        std::fprintf(stderr, "a format path was not exercised\n");
        return 1;
    }
    std::printf("zstd host encoder: %llu frames decoded exactly by %s\n",
                (unsigned long long)frames, libp);
    return 0;
}
