// zstd_lab -- ratio lab for the device zstd encoder (dev tool, not product).
//
// A serial encoder over the format pieces of csrc/aqz_zstd.hh with the
// knobs the device encoder could take: parse window / unit, hash-chain depth,
// lazy matching, minimum match, repeat offsets, Huffman table scope,
// predefined vs custom FSE sequence tables, and the far candidates of
// zstd_far (far=<log2 table entries>, farbatch, fartag, farmin, farcap,
// farcost).  Every frame is decoded by libzstd and compared; sizes are set
// against libzstd's levels on the same payloads (camera-like and dim sCMOS
// u16: plain 8 MiB chunks, byte-shuffled (_shuf) and bitshuffled (_bit)
// 256 KiB blosc blocks).
//
//   hipcc -x hip --cuda-host-only -std=c++20 -O2 -I acquire-zarr_amd/csrc \
//         tools/zstd_lab.cpp -ldl -o tools/zstd_lab
//   tools/zstd_lab /opt/conda/lib/libzstd.so.1 [key=value ...]
#include "aqz_zstd.hh"

#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <vector>

using namespace aqz::zstd;

namespace {

struct Opt
{
    uint32_t block = kBlock;  // zstd block content
    uint32_t unit = 4096;     // parse unit (matches end inside it)
    uint32_t hist = 0;        // bytes before the unit a match may reach
    uint32_t window = 1u << 22;
    uint32_t minmatch = 4;
    int entropy_min = 1;      // the device's entropy rule for the min match
    double match_bits = 16.0;
    uint32_t chain = 1;       // candidates per position (1 = single table)
    int lazy = 0;
    int rep = 0;              // repeat offsets
    int reprobe = 1;          // the parse tries the repeat offsets at each position
    int huf = 0;              // 0 frame table, 1 per block, 2 adaptive
    int seqtab = 0;           // 0 predefined, 1 custom per frame, 2 per block (repeat allowed)
    int hashlog = 12;
    uint32_t hufgroup = 8;    // huf=4: blocks per Huffman table group
    // far candidates (the device's zstd_far model): a table of 2^far entries
    // over the whole segment, most recent position per bucket with a tag,
    // probed and then filled in batches of farbatch positions; a far match
    // needs farmin bytes
    int far = 0;
    uint32_t farmin = 5;
    uint32_t farbatch = 256;
    uint32_t fartag = 9;
    int farcost = 0;          // 1: the device's cost rule for far matches
    uint32_t farcap = 1u << 30; // far match bytes measured
};
double g_H = 8.0; // the block's byte entropy (parse_block)

// far[i] = candidate position for segment position i (-1: none), keyed on
// the 5 bytes at i
std::vector<int64_t> g_far;

std::map<std::string, double> g_stats;

// ---- FSE normalisation -----------------------------------------------------
// counts -> norm summing to 1 << al (-1 = "less than 1"); false if impossible
bool
normalize(const uint32_t* cnt, uint32_t maxsym, uint32_t al, int16_t* norm)
{
    uint64_t total = 0;
    for (uint32_t s = 0; s <= maxsym; ++s)
        total += cnt[s];
    if (total == 0)
        return false;
    const int ts = 1 << al;
    int used = 0, big = -1;
    for (uint32_t s = 0; s <= maxsym; ++s) {
        if (!cnt[s]) {
            norm[s] = 0;
            continue;
        }
        const double p = double(cnt[s]) * ts / double(total);
        if (p < 1.0) {
            norm[s] = -1;
            used += 1;
        } else {
            int v = int(p + 0.5);
            norm[s] = int16_t(v);
            used += v;
        }
        if (big < 0 || cnt[s] > cnt[big])
            big = int(s);
    }
    const int fix = norm[big] + (ts - used);
    if (norm[big] < 0 || fix < 1)
        return false;
    norm[big] = int16_t(fix);
    return true;
}

double
cost_bits(const uint32_t* cnt, uint32_t maxsym, const int16_t* norm, uint32_t al)
{
    double b = 0;
    for (uint32_t s = 0; s <= maxsym; ++s) {
        if (!cnt[s])
            continue;
        if (norm[s] == 0)
            return 1e30; // not encodable
        const double p = norm[s] < 0 ? 1.0 : double(norm[s]);
        b += cnt[s] * (al - std::log2(p));
    }
    return b;
}

struct SeqTab
{
    FseTable<kSeqMaxLog> ct;
    int16_t norm[kFseMaxSym];
    uint32_t maxsym = 0, al = 0;
    bool valid = false;
};

// ---- parse -----------------------------------------------------------------
struct Seq3
{
    uint32_t lit, len, off; // off = actual distance
};

struct Parsed
{
    std::vector<Seq3> seqs;
    std::vector<uint8_t> lits;
};

// one block [b0, b1) of src; matches may reach back to
// max(0, p - window, unit start - hist) and end inside the unit
Parsed
parse_block(const uint8_t* src, uint64_t b0, uint64_t b1, const Opt& o, const uint32_t* rep_in)
{
    Parsed out;
    const uint32_t HL = uint32_t(o.hashlog);
    std::vector<int64_t> head(size_t(1) << HL, -1);
    std::vector<int64_t> prev(b1 - b0 + o.hist + o.unit + 8, -1);
    auto rd4 = [&](uint64_t p) {
        uint32_t v;
        std::memcpy(&v, src + p, 4);
        return v;
    };
    auto hsh = [&](uint64_t p) { return (rd4(p) * 2654435761u) >> (32 - HL); };
    // entropy-based minimum match of the device (per block)
    uint32_t minlen = o.minmatch;
    if (o.entropy_min) {
        uint32_t h256[256] = { 0 };
        for (uint64_t i = b0; i < b1; ++i)
            h256[src[i]]++;
        double H = 0;
        const double n = double(b1 - b0);
        for (int k = 0; k < 256; ++k)
            if (h256[k])
                H -= h256[k] / n * std::log2(h256[k] / n);
        minlen = std::max<uint32_t>(o.minmatch,
                                    uint32_t(std::ceil(o.match_bits / std::max(H, 0.25))));
        minlen = std::min<uint32_t>(minlen, 64);
        g_H = std::max(H, 0.25);
    }
    // insert history positions
    const uint64_t base = b0 >= o.hist ? b0 - o.hist : 0;
    auto pidx = [&](uint64_t p) { return size_t(p - base); };
    prev.assign(b1 - base + 8, -1);
    auto insert = [&](uint64_t p) {
        if (p + 4 > b1)
            return;
        const uint32_t h = hsh(p);
        prev[pidx(p)] = head[h];
        head[h] = int64_t(p);
    };
    uint64_t unit0 = b0;
    for (uint64_t p = base; p < b0; ++p)
        insert(p);
    uint32_t rep[3] = { rep_in[0], rep_in[1], rep_in[2] };
    uint32_t known = 0; // rep slots set inside this block (see to_codes)
    uint64_t anchor = b0, p = b0;
    auto lo_of = [&](uint64_t q) {
        const uint64_t us = q - ((q - b0) % o.unit); // unit start (units tile the block)
        uint64_t lo = us >= o.hist ? us - o.hist : 0;
        if (q > o.window)
            lo = std::max<uint64_t>(lo, q - o.window);
        return lo;
    };
    auto unit_end = [&](uint64_t q) { return std::min<uint64_t>(b1, q - ((q - b0) % o.unit) + o.unit); };
    auto match_len = [&](uint64_t a, uint64_t q, uint64_t end) {
        uint32_t l = 0;
        while (q + l < end && src[a + l] == src[q + l])
            ++l;
        return l;
    };
    struct Best
    {
        uint32_t len = 0, off = 0;
        bool isrep = false;
    };
    auto find = [&](uint64_t q) {
        Best b;
        if (q + 4 > b1)
            return b;
        const uint64_t lo = lo_of(q), end = unit_end(q);
        if (o.rep && o.reprobe) {
            const uint32_t ll = uint32_t(q - anchor);
            for (int k = 0; k < int(known); ++k) {
                const uint32_t r = rep[k];
                if (k == 0 && ll == 0)
                    continue; // rep0 with LL=0 is not a repeat code
                if (r == 0 || r > q - lo)
                    continue;
                const uint32_t l = match_len(q - r, q, end);
                if (l >= 3 && l > b.len) {
                    b = Best{ l, r, true };
                }
            }
        }
        if (o.far && !g_far.empty() && g_far[q] >= 0 && !o.farcost) {
            const uint64_t c = uint64_t(g_far[q]);
            const uint32_t l = std::min<uint32_t>(match_len(c, q, end), o.farcap);
            if (l >= o.farmin && l > b.len + (b.isrep ? 1 : 0))
                b = Best{ l, uint32_t(q - c), false };
        }
        int64_t c = head[hsh(q)];
        for (uint32_t d = 0; d < o.chain && c >= 0; ++d) {
            if (uint64_t(c) >= lo && uint64_t(c) < q) {
                const uint32_t l = match_len(uint64_t(c), q, end);
                // a repcode match wins ties within 1 byte (cheaper offset)
                if (l > b.len + (b.isrep ? 1 : 0)) {
                    b = Best{ l, uint32_t(q - uint64_t(c)), false };
                }
            } else if (uint64_t(c) < lo) {
                break;
            }
            c = prev[pidx(uint64_t(c))];
        }
        const uint32_t need = b.isrep ? 3u : (o.far && b.off > q - lo_of(q)) ? o.farmin : minlen;
        if (b.len < need)
            b.len = 0;
        if (o.far && o.farcost && !g_far.empty() && g_far[q] >= 0) {
            // the device rule: a far match pays its extra offset bits
            const uint64_t c = uint64_t(g_far[q]);
            const uint32_t l = std::min<uint32_t>(match_len(c, q, end), 16);
            const uint32_t d = uint32_t(q - c);
            const double fob = std::floor(std::log2(double(d) + 3));
            bool take = l >= o.farmin && l * g_H >= o.match_bits + fob - 10.0;
            if (take && b.len)
                take = (double(l) - b.len) * g_H > fob - std::floor(std::log2(double(b.off) + 3));
            if (take)
                b = Best{ l, d, false };
        }
        return b;
    };
    (void)unit0;
    while (p + 4 <= b1) {
        Best b = find(p);
        if (b.len && o.lazy) {
            insert(p);
            Best n = find(p + 1);
            if (n.len > b.len + 1 || (n.len > b.len && n.isrep)) {
                ++p;
                b = n;
            }
        } else {
            insert(p);
        }
        if (!b.len) {
            ++p;
            continue;
        }
        out.seqs.push_back(Seq3{ uint32_t(p - anchor), b.len, b.off });
        out.lits.insert(out.lits.end(), src + anchor, src + p);
        // repcode history (actual offsets, MRU of distinct values)
        if (b.off == rep[0]) {
        } else if (b.off == rep[1]) {
            std::swap(rep[0], rep[1]);
        } else if (b.off == rep[2]) {
            const uint32_t t = rep[2];
            rep[2] = rep[1];
            rep[1] = rep[0];
            rep[0] = t;
        } else {
            rep[2] = rep[1];
            rep[1] = rep[0];
            rep[0] = b.off;
            known = known < 3 ? known + 1 : 3;
        }
        for (uint64_t q = p + 1; q < p + b.len; ++q)
            insert(q);
        p += b.len;
        anchor = p;
    }
    out.lits.insert(out.lits.end(), src + anchor, src + b1);
    return out;
}

// ---- sequences with repeat codes -------------------------------------------
struct SeqCode
{
    uint32_t lit, len, ofv; // ofv: zstd Offset_Value (1..3 repeat, else off + 3)
};

// actual offsets -> Offset_Values under the decoder's repeat rules (RFC
// 8878 3.1.2.5); rep is the running history, updated
// Repeat codes only ever reference history slots set by this block's own
// earlier sequences (`known` of them): a block's coding is then independent
// of the blocks before it -- of whether they were emitted raw, RLE or
// compressed -- which is what lets the device encode blocks in parallel.
std::vector<SeqCode>
to_codes(const std::vector<Seq3>& s, uint32_t* rep, bool use_rep)
{
    std::vector<SeqCode> out;
    uint32_t known = 0;
    for (const Seq3& q : s) {
        uint32_t ofv = q.off + 3;
        int kind = -1; // 0..2 rep index, 3 = rep0 - 1
        if (use_rep) {
            if (q.lit > 0) {
                for (uint32_t k = 0; k < known && kind < 0; ++k)
                    if (q.off == rep[k]) {
                        kind = int(k);
                        ofv = k + 1;
                    }
            } else {
                if (known > 1 && q.off == rep[1]) {
                    kind = 1;
                    ofv = 1;
                } else if (known > 2 && q.off == rep[2]) {
                    kind = 2;
                    ofv = 2;
                } else if (known > 0 && rep[0] > 1 && q.off == rep[0] - 1) {
                    kind = 3;
                    ofv = 3;
                }
            }
        }
        if (kind < 0 || kind == 3)
            known = known < 3 ? known + 1 : 3;
        if (kind < 0 || kind == 3) {
            rep[2] = rep[1];
            rep[1] = rep[0];
            rep[0] = q.off;
        } else if (kind == 1) {
            std::swap(rep[0], rep[1]);
        } else if (kind == 2) {
            const uint32_t t = rep[2];
            rep[2] = rep[1];
            rep[1] = rep[0];
            rep[0] = t;
        }
        out.push_back(SeqCode{ q.lit, q.len, ofv });
    }
    return out;
}

template<class TL, class TO, class TM>
uint32_t
encode_seq_codes(const TL& tl, const TO& to, const TM& tm, const std::vector<SeqCode>& v,
                 uint8_t* out, uint32_t cap)
{
    BitW w;
    w.init(out, cap);
    const uint32_t n = uint32_t(v.size());
    SeqCode z = v[n - 1];
    uint32_t llc = ll_code(z.lit), mlc = ml_code(z.len), ofc = highbit(z.ofv);
    uint32_t sml = fse_init(tm, mlc), sof = fse_init(to, ofc), sll = fse_init(tl, llc);
    w.add(z.lit - ll_base(llc), ll_bits(llc));
    w.add(z.len - ml_base(mlc), ml_bits(mlc));
    w.add(z.ofv - (1u << ofc), ofc);
    for (int i = int(n) - 2; i >= 0; --i) {
        z = v[size_t(i)];
        llc = ll_code(z.lit);
        mlc = ml_code(z.len);
        ofc = highbit(z.ofv);
        fse_enc(w, sof, to, ofc);
        fse_enc(w, sml, tm, mlc);
        fse_enc(w, sll, tl, llc);
        w.add(z.lit - ll_base(llc), ll_bits(llc));
        w.add(z.len - ml_base(mlc), ml_bits(mlc));
        w.add(z.ofv - (1u << ofc), ofc);
    }
    fse_flush(w, sml, tm);
    fse_flush(w, sof, to);
    fse_flush(w, sll, tl);
    return w.close();
}

// ---- Huffman ---------------------------------------------------------------
struct Huf
{
    int mode = 0; // 0 none, 1 single symbol, 2 table
    uint8_t len[256];
    uint16_t code[256];
    uint8_t tree[160];
    uint32_t tree_n = 0;
};

Huf
make_huf(const uint32_t* hist)
{
    Huf t;
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

uint32_t
huf_streams(const Huf& t, const uint8_t* lit, uint32_t n, uint8_t* out, uint32_t cap)
{
    const uint32_t seg = lit_segment(n);
    uint32_t at = 6, sz[4];
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t a = std::min(n, k * seg), b = std::min(n, (k + 1) * seg);
        for (uint32_t i = a; i < b; ++i)
            if (!t.len[lit[i]])
                return 0; // symbol absent from this table
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

// ---- frame -----------------------------------------------------------------
struct FrameStats
{
    uint64_t lit_bytes = 0, seq_bytes = 0, hdr = 0, raw_blocks = 0, nseq = 0, nlit = 0,
             rep_codes = 0, tables = 0;
};

std::vector<uint8_t>
encode_frame(const uint8_t* src, uint64_t n, const Opt& o, FrameStats& fs)
{
    std::vector<uint8_t> out(frame_header_bytes(n) + n + 3 * (n / o.block + 1) + 1024);
    uint32_t at = write_frame_header(out.data(), n);
    const uint32_t nb = uint32_t((n + o.block - 1) / o.block);
    uint32_t rep_parse[3] = { 1, 4, 8 };
    std::vector<Parsed> P(nb);
    g_far.clear();
    if (o.far) {
        g_far.assign(n, -1);
        const uint32_t FL = uint32_t(o.far), TB = o.fartag;
        std::vector<uint32_t> tab(size_t(1) << FL, 0); // (pos + 1) << TB | tag
        auto key = [&](uint64_t i) {
            uint64_t k = 0;
            std::memcpy(&k, src + i, 5);
            return (k * 0x9E3779B97F4A7C15ull) >> (64 - FL - TB);
        };
        const uint64_t last = n >= 5 ? n - 5 : 0;
        for (uint64_t b = 0; b + 5 <= n; b += o.farbatch) {
            const uint64_t e = std::min<uint64_t>(last + 1, b + o.farbatch);
            for (uint64_t i = b; i < e; ++i) { // probe
                const uint64_t h = key(i);
                const uint32_t v = tab[h >> TB];
                if (v && (v & ((1u << TB) - 1)) == (h & ((1u << TB) - 1)))
                    g_far[i] = int64_t(v >> TB) - 1;
            }
            for (uint64_t i = b; i < e; ++i) { // insert (the latest wins)
                const uint64_t h = key(i);
                tab[h >> TB] = uint32_t(((i + 1) << TB) | (h & ((1u << TB) - 1)));
            }
        }
    }
    uint32_t fhist[256] = { 0 };
    for (uint32_t j = 0; j < nb; ++j) {
        const uint64_t b0 = uint64_t(j) * o.block, b1 = std::min<uint64_t>(n, b0 + o.block);
        P[j] = parse_block(src, b0, b1, o, rep_parse);
        // the parse's own rep history follows the sequences
        uint32_t r[3] = { rep_parse[0], rep_parse[1], rep_parse[2] };
        (void)to_codes(P[j].seqs, r, true);
        std::memcpy(rep_parse, r, sizeof r);
        for (uint8_t x : P[j].lits)
            fhist[x]++;
    }
    const Huf ftab = make_huf(fhist);
    // huf=4: one table per group of hufgroup blocks
    std::vector<Huf> gtab;
    if (o.huf == 4) {
        for (uint32_t g0 = 0; g0 < nb; g0 += o.hufgroup) {
            uint32_t gh[256] = { 0 };
            for (uint32_t j = g0; j < std::min(nb, g0 + o.hufgroup); ++j)
                for (uint8_t x : P[j].lits)
                    gh[x]++;
            gtab.push_back(make_huf(gh));
        }
    }
    // frame-scope custom sequence tables
    uint32_t rep[3] = { 1, 4, 8 };
    std::vector<std::vector<SeqCode>> codes(nb);
    uint32_t fll[64] = { 0 }, fof[64] = { 0 }, fml[64] = { 0 };
    for (uint32_t j = 0; j < nb; ++j) {
        codes[j] = to_codes(P[j].seqs, rep, o.rep != 0);
        for (const SeqCode& c : codes[j]) {
            fll[ll_code(c.lit)]++;
            fof[highbit(c.ofv)]++;
            fml[ml_code(c.len)]++;
        }
    }
    FseTable<kSeqMaxLog> dll, dof, dml;
    fse_build(dll, ll_default_norm(), 35, 6);
    fse_build(dml, ml_default_norm(), 52, 6);
    fse_build(dof, of_default_norm(), 28, 5);
    auto make_tab = [&](const uint32_t* cnt, uint32_t maxsym_cap, uint32_t maxlog, SeqTab& t) {
        uint32_t ms = 0, nz = 0;
        uint64_t tot = 0;
        for (uint32_t s = 0; s <= maxsym_cap; ++s)
            if (cnt[s]) {
                ms = s;
                ++nz;
                tot += cnt[s];
            }
        t.valid = false;
        if (nz < 1)
            return;
        double bestc = 1e30;
        for (uint32_t al = 5; al <= maxlog; ++al) {
            int16_t nm[kFseMaxSym];
            if (!normalize(cnt, ms, al, nm))
                continue;
            uint8_t tmp[512];
            const uint32_t d = fse_write_ncount(tmp, sizeof tmp, nm, ms, al);
            if (!d)
                continue;
            const double c = cost_bits(cnt, ms, nm, al) + 8.0 * d;
            if (c < bestc) {
                bestc = c;
                std::memcpy(t.norm, nm, sizeof nm);
                t.al = al;
                t.maxsym = ms;
            }
        }
        if (bestc < 1e29)
            t.valid = fse_build(t.ct, t.norm, t.maxsym, t.al);
        (void)tot;
    };
    SeqTab Fll, Fof, Fml;
    if (o.seqtab == 1) {
        make_tab(fll, 35, 9, Fll);
        make_tab(fof, 31, 8, Fof);
        make_tab(fml, 52, 9, Fml);
    }
    bool frame_tabs_sent = false;
    // per-block repeat state of custom tables
    SeqTab Pll, Pof, Pml; // last tables in force (mode 2 per-block)
    bool have_prev = false;
    const Huf* last_huf = nullptr;
    Huf blk_huf;
    std::vector<uint8_t> tmp(2 * o.block + 4096);
    for (uint32_t j = 0; j < nb; ++j) {
        const uint64_t b0 = uint64_t(j) * o.block, b1 = std::min<uint64_t>(n, b0 + o.block);
        const uint32_t bn = uint32_t(b1 - b0);
        const bool last = j + 1 == nb;
        const uint8_t* b = src + b0;
        bool same = true;
        for (uint32_t i = 1; i < bn && same; ++i)
            same = b[i] == b[0];
        if (same) {
            write_block_header(out.data() + at, last, 1, bn);
            out[at + 3] = b[0];
            at += 4;
            fs.hdr += 4;
            continue;
        }
        const std::vector<uint8_t>& L = P[j].lits;
        const uint32_t nl = uint32_t(L.size());
        // ---- literals: candidates
        uint32_t lsz = 0;
        const Huf* used = nullptr;
        {
            bool lsame = nl > 0;
            for (uint32_t i = 1; i < nl && lsame; ++i)
                lsame = L[i] == L[0];
            std::vector<uint8_t> best;
            uint32_t best_n = nl + lit_header_raw_bytes(nl);
            int best_kind = 0; // 0 raw, 1 rle, 2 new tree, 3 treeless
            const Huf* best_tab = nullptr;
            if (lsame && nl >= 2) {
                best_kind = 1;
                best_n = lit_header_raw_bytes(nl) + 1;
            } else if (nl >= 64) {
                auto try_tab = [&](const Huf& t, bool with_tree) {
                    if (t.mode != 2)
                        return;
                    std::vector<uint8_t> s(nl + nl / 2 + 64);
                    const uint32_t sn = huf_streams(t, L.data(), nl, s.data(), uint32_t(s.size()));
                    if (!sn)
                        return;
                    const uint32_t cs = (with_tree ? t.tree_n : 0) + sn;
                    const uint32_t tot = lit_header_huf_bytes(nl, cs) + cs;
                    if (tot < best_n) {
                        best_n = tot;
                        best_kind = with_tree ? 2 : 3;
                        best_tab = &t;
                        best = std::move(s);
                        best.resize(sn);
                    }
                };
                if (o.huf == 0) {
                    try_tab(ftab, last_huf == nullptr);
                } else if (o.huf == 4) {
                    const Huf& gt = gtab[j / o.hufgroup];
                    try_tab(gt, last_huf != &gt);
                } else if (o.huf == 3) {
                    // own tree, or the segment's table (treeless while the
                    // decoder's last table is it, else carried again)
                    uint32_t h[256] = { 0 };
                    for (uint8_t x : L)
                        h[x]++;
                    blk_huf = make_huf(h);
                    try_tab(blk_huf, true);
                    try_tab(ftab, last_huf != &ftab);
                } else {
                    uint32_t h[256] = { 0 };
                    for (uint8_t x : L)
                        h[x]++;
                    blk_huf = make_huf(h);
                    if (o.huf == 1 || !last_huf)
                        try_tab(blk_huf, true);
                    else {
                        try_tab(blk_huf, true);
                        try_tab(*last_huf, false);
                    }
                }
            }
            if (best_kind == 1) {
                lsz = write_lit_header_raw(tmp.data(), 1, nl);
                tmp[lsz++] = L[0];
            } else if (best_kind >= 2) {
                const uint32_t cs = (best_kind == 2 ? best_tab->tree_n : 0) + uint32_t(best.size());
                lsz = write_lit_header_huf(tmp.data(), best_kind == 2 ? 2 : 3, nl, cs);
                if (best_kind == 2) {
                    std::memcpy(tmp.data() + lsz, best_tab->tree, best_tab->tree_n);
                    lsz += best_tab->tree_n;
                }
                std::memcpy(tmp.data() + lsz, best.data(), best.size());
                lsz += uint32_t(best.size());
                used = best_tab;
            } else {
                lsz = write_lit_header_raw(tmp.data(), 0, nl);
                std::memcpy(tmp.data() + lsz, L.data(), nl);
                lsz += nl;
            }
        }
        // ---- sequences
        const std::vector<SeqCode>& sc = codes[j];
        uint32_t csz = lsz;
        const uint32_t ns = uint32_t(sc.size());
        SeqTab Bll, Bof, Bml; // this block's choice
        int mll = 0, mof = 0, mml = 0;
        if (ns == 0) {
            tmp[csz++] = 0;
        } else {
            uint32_t cll[64] = { 0 }, cof[64] = { 0 }, cml[64] = { 0 };
            for (const SeqCode& c : sc) {
                cll[ll_code(c.lit)]++;
                cof[highbit(c.ofv)]++;
                cml[ml_code(c.len)]++;
            }
            // header
            uint32_t k = 0;
            uint8_t* h = tmp.data() + csz;
            if (ns < 128) {
                h[0] = uint8_t(ns);
                k = 1;
            } else if (ns < 0x7F00) {
                h[0] = uint8_t((ns >> 8) + 0x80);
                h[1] = uint8_t(ns);
                k = 2;
            } else {
                h[0] = 0xFF;
                put_le(h + 1, ns - 0x7F00, 2);
                k = 3;
            }
            uint8_t* modes = h + k;
            csz += k + 1;
            // choose a mode per table: 0 predefined, 2 compressed, 3 repeat
            auto choose = [&](const uint32_t* cnt, uint32_t cap_sym, uint32_t maxlog,
                              const int16_t* defn, uint32_t defmax, uint32_t defal,
                              const SeqTab& frame_t, const SeqTab& prev_t, SeqTab& outt,
                              int& mode) {
                double c0 = cost_bits(cnt, defmax, defn, defal);
                for (uint32_t s = defmax + 1; s <= cap_sym; ++s)
                    if (cnt[s])
                        c0 = 1e30;
                mode = 0;
                double best = c0;
                if (o.seqtab == 1 && frame_t.valid) {
                    const double c = cost_bits(cnt, frame_t.maxsym, frame_t.norm, frame_t.al);
                    bool cover = true;
                    for (uint32_t s = frame_t.maxsym + 1; s <= cap_sym; ++s)
                        cover &= cnt[s] == 0;
                    if (cover) {
                        // the table is described once per frame; later blocks repeat it
                        uint8_t t2[512];
                        const uint32_t d = frame_tabs_sent ? 0
                                                           : fse_write_ncount(t2, sizeof t2,
                                                                              frame_t.norm,
                                                                              frame_t.maxsym,
                                                                              frame_t.al);
                        if (c + 8.0 * d < best) {
                            best = c + 8.0 * d;
                            mode = frame_tabs_sent ? 3 : 2;
                            outt = frame_t;
                        }
                    }
                }
                if (o.seqtab >= 2) {
                    SeqTab t;
                    make_tab(cnt, cap_sym, maxlog, t);
                    if (t.valid) {
                        uint8_t t2[512];
                        const uint32_t d = fse_write_ncount(t2, sizeof t2, t.norm, t.maxsym, t.al);
                        const double c = cost_bits(cnt, t.maxsym, t.norm, t.al) + 8.0 * d;
                        if (c < best) {
                            best = c;
                            mode = 2;
                            outt = t;
                        }
                    }
                    if (o.seqtab == 2 && have_prev && prev_t.valid) {
                        bool cover = true;
                        for (uint32_t s = prev_t.maxsym + 1; s <= cap_sym; ++s)
                            cover &= cnt[s] == 0;
                        const double c = cover ? cost_bits(cnt, prev_t.maxsym, prev_t.norm,
                                                           prev_t.al)
                                               : 1e30;
                        if (c < best) {
                            best = c;
                            mode = 3;
                            outt = prev_t;
                        }
                    }
                }
            };
            if (o.seqtab == 1) {
                // the segment's tables for every block: described by the
                // first block with sequences, repeated by the rest
                if (Fll.valid && Fof.valid && Fml.valid) {
                    mll = mof = mml = frame_tabs_sent ? 3 : 2;
                    Bll = Fll;
                    Bof = Fof;
                    Bml = Fml;
                }
            } else {
                choose(cll, 35, 9, ll_default_norm(), 35, 6, Fll, Pll, Bll, mll);
                choose(cof, 31, 8, of_default_norm(), 28, 5, Fof, Pof, Bof, mof);
                choose(cml, 52, 9, ml_default_norm(), 52, 6, Fml, Pml, Bml, mml);
            }
            *modes = uint8_t(mll << 6 | mof << 4 | mml << 2);
            auto desc = [&](int mode, const SeqTab& t) {
                if (mode == 2) {
                    const uint32_t d = fse_write_ncount(tmp.data() + csz, 512, t.norm, t.maxsym,
                                                        t.al);
                    csz += d;
                    fs.tables += d;
                }
            };
            desc(mll, Bll);
            desc(mof, Bof);
            desc(mml, Bml);
            FseTable<kSeqMaxLog> ull, uof, uml;
            auto pick = [&](int mode, const SeqTab& t, const FseTable<kSeqMaxLog>& def,
                            FseTable<kSeqMaxLog>& u) {
                if (mode == 0)
                    u = def;
                else
                    u = t.ct;
            };
            pick(mll, Bll, dll, ull);
            pick(mof, Bof, dof, uof);
            pick(mml, Bml, dml, uml);
            const uint32_t q = encode_seq_codes(ull, uof, uml, sc, tmp.data() + csz,
                                                uint32_t(tmp.size()) - csz);
            if (!q) {
                fprintf(stderr, "seq overflow\n");
                exit(3);
            }
            csz += q;
        }
        if (csz >= bn) {
            write_block_header(out.data() + at, last, 0, bn);
            std::memcpy(out.data() + at + 3, b, bn);
            at += 3 + bn;
            fs.raw_blocks++;
            fs.hdr += 3;
            continue;
        }
        // committed: update the entropy state the decoder keeps
        if (used) {
            if (o.huf == 4)
                last_huf = used;
            else if (o.huf == 0 || used == &ftab)
                last_huf = &ftab;
            else if (used == &blk_huf) {
                static Huf keep[2];
                static int ki = 0;
                keep[ki] = blk_huf;
                last_huf = &keep[ki];
                ki ^= 1;
            }
        }
        if (ns) {
            if (o.seqtab == 1 && (mll == 2 || mof == 2 || mml == 2))
                frame_tabs_sent = true;
            if (mll)
                Pll = Bll;
            else
                Pll.valid = false;
            if (mof)
                Pof = Bof;
            else
                Pof.valid = false;
            if (mml)
                Pml = Bml;
            else
                Pml.valid = false;
            have_prev = true;
            fs.nseq += ns;
            for (const SeqCode& c : sc)
                fs.rep_codes += c.ofv <= 3;
        }
        fs.nlit += nl;
        fs.lit_bytes += lsz;
        fs.seq_bytes += csz - lsz;
        fs.hdr += 3;
        write_block_header(out.data() + at, last, 2, csz);
        std::memcpy(out.data() + at + 3, tmp.data(), csz);
        at += 3 + csz;
    }
    out.resize(at);
    return out;
}

using dec_t = size_t (*)(void*, size_t, const void*, size_t);
using err_t = unsigned (*)(size_t);
using name_t = const char* (*)(size_t);
using cmp_t = size_t (*)(void*, size_t, const void*, size_t, int);

std::vector<uint8_t>
payload(const std::string& kind, uint64_t n, uint32_t seed)
{
    std::mt19937 rng(seed);
    std::vector<uint8_t> v(n);
    const uint64_t np = n / 2;
    std::vector<uint16_t> px(np);
    const bool dim = kind.rfind("dim", 0) == 0;
    std::normal_distribution<double> nd(0.0, dim ? 3.0 : 30.0);
    for (uint64_t i = 0; i < np; ++i) {
        const double base = dim ? 100.0 : 1000 + 200 * std::sin(double(i) / 977.0);
        px[i] = uint16_t(std::clamp(base + nd(rng), 0.0, 65535.0));
    }
    if (kind.find("bit") != std::string::npos) { // bitshuffle in 256 KiB blosc blocks
        for (uint64_t b0 = 0; b0 < np; b0 += 131072) {
            const uint64_t m = std::min<uint64_t>(131072, np - b0);
            uint8_t* o = v.data() + 2 * b0;
            std::memset(o, 0, 2 * m);
            for (uint64_t i = 0; i < m; ++i)
                for (int bit = 0; bit < 16; ++bit)
                    if ((px[b0 + i] >> bit) & 1)
                        o[bit * (m / 8) + i / 8] |= uint8_t(1u << (i % 8));
        }
    } else if (kind.find("shuf") == std::string::npos) {
        std::memcpy(v.data(), px.data(), 2 * np);
    } else { // byte shuffle in 256 KiB blosc blocks
        for (uint64_t b0 = 0; b0 < np; b0 += 131072) {
            const uint64_t m = std::min<uint64_t>(131072, np - b0);
            for (uint64_t i = 0; i < m; ++i) {
                v[2 * b0 + i] = uint8_t(px[b0 + i]);
                v[2 * b0 + m + i] = uint8_t(px[b0 + i] >> 8);
            }
        }
    }
    return v;
}

} // namespace

int
main(int argc, char** argv)
{
    void* h = dlopen(argc > 1 ? argv[1] : "libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h)
        return 2;
    auto dec = reinterpret_cast<dec_t>(dlsym(h, "ZSTD_decompress"));
    auto iserr = reinterpret_cast<err_t>(dlsym(h, "ZSTD_isError"));
    auto ename = reinterpret_cast<name_t>(dlsym(h, "ZSTD_getErrorName"));
    auto cmp = reinterpret_cast<cmp_t>(dlsym(h, "ZSTD_compress"));
    Opt o;
    std::string kinds = "camera,dim,camera_shuf,dim_shuf";
    int ref = 1;
    uint64_t chunk = 8 << 20;
    for (int i = 2; i < argc; ++i) {
        std::string a = argv[i];
        const auto e = a.find('=');
        const std::string k = a.substr(0, e);
        const std::string v = e == std::string::npos ? "1" : a.substr(e + 1);
        const long x = std::atol(v.c_str());
        if (k == "block") o.block = uint32_t(x);
        else if (k == "unit") o.unit = uint32_t(x);
        else if (k == "hist") o.hist = uint32_t(x);
        else if (k == "window") o.window = uint32_t(x);
        else if (k == "minmatch") o.minmatch = uint32_t(x);
        else if (k == "entropy") o.entropy_min = int(x);
        else if (k == "mbits") o.match_bits = std::atof(v.c_str());
        else if (k == "chain") o.chain = uint32_t(x);
        else if (k == "lazy") o.lazy = int(x);
        else if (k == "rep") o.rep = int(x);
        else if (k == "reprobe") o.reprobe = int(x);
        else if (k == "huf") o.huf = int(x);
        else if (k == "seqtab") o.seqtab = int(x);
        else if (k == "hashlog") o.hashlog = int(x);
        else if (k == "hufgroup") o.hufgroup = uint32_t(x);
        else if (k == "far") o.far = int(x);
        else if (k == "farmin") o.farmin = uint32_t(x);
        else if (k == "farbatch") o.farbatch = uint32_t(x);
        else if (k == "fartag") o.fartag = uint32_t(x);
        else if (k == "farcost") o.farcost = int(x);
        else if (k == "farcap") o.farcap = uint32_t(x);
        else if (k == "kinds") kinds = v;
        else if (k == "ref") ref = int(x);
        else if (k == "chunk") chunk = uint64_t(x);
        else {
            fprintf(stderr, "unknown option %s\n", k.c_str());
            return 2;
        }
    }
    size_t p0 = 0;
    while (p0 < kinds.size()) {
        size_t p1 = kinds.find(',', p0);
        if (p1 == std::string::npos)
            p1 = kinds.size();
        const std::string kind = kinds.substr(p0, p1 - p0);
        p0 = p1 + 1;
        const bool shuf = kind.find("shuf") != std::string::npos || kind.find("bit") != std::string::npos;
        const std::vector<uint8_t> src = payload(kind, chunk, 7);
        const uint64_t seg = shuf ? (256u << 10) : chunk; // one frame per segment
        uint64_t ours = 0;
        FrameStats fs;
        uint64_t refb[4] = { 0, 0, 0, 0 };
        const int levels[4] = { 1, 3, 5, 9 };
        for (uint64_t s0 = 0; s0 < chunk; s0 += seg) {
            const uint64_t sn = std::min(seg, chunk - s0);
            const std::vector<uint8_t> f = encode_frame(src.data() + s0, sn, o, fs);
            std::vector<uint8_t> back(sn + 16);
            const size_t r = dec(back.data(), back.size(), f.data(), f.size());
            if (iserr(r) || r != sn || std::memcmp(back.data(), src.data() + s0, sn)) {
                fprintf(stderr, "DECODE FAIL %s seg %llu: %s\n", kind.c_str(),
                        (unsigned long long)s0, iserr(r) ? ename(r) : "mismatch");
                return 1;
            }
            ours += f.size();
            if (ref)
                for (int l = 0; l < 4; ++l) {
                    std::vector<uint8_t> z(sn + sn / 64 + 1024);
                    const size_t zn = cmp(z.data(), z.size(), src.data() + s0, sn, levels[l]);
                    refb[l] += iserr(zn) ? sn : zn;
                }
        }
        printf("%-12s ours %9llu (ratio %6.3f) lit %llu seq %llu tab %llu nseq %llu rep %llu "
               "nlit %llu raw %llu",
               kind.c_str(), (unsigned long long)ours, double(chunk) / ours,
               (unsigned long long)fs.lit_bytes, (unsigned long long)fs.seq_bytes,
               (unsigned long long)fs.tables, (unsigned long long)fs.nseq,
               (unsigned long long)fs.rep_codes, (unsigned long long)fs.nlit,
               (unsigned long long)fs.raw_blocks);
        if (ref)
            printf(" | zstd1 %.3f zstd3 %.3f zstd5 %.3f zstd9 %.3f | ours/z5 %.3f ours/z9 %.3f",
                   double(chunk) / refb[0], double(chunk) / refb[1], double(chunk) / refb[2],
                   double(chunk) / refb[3], double(ours) / refb[2], double(ours) / refb[3]);
        printf("\n");
        fflush(stdout);
    }
    return 0;
}
