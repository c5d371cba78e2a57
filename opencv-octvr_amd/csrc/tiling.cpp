// tiling.cpp — the tiled composite LUT (kernels.hpp "tiled composite"), built once per rig.
//
// A job is one 128 x (8 qpl) output tile written by one launch item (qpl = 2 for the blend = 0
// composite: each lane of the workgroup takes two quads, halving the per-item costs per pixel): for blend = 0 every tile of the output
// frame (each pixel's entry = the winning camera of the copy chain), for blend > 0 every level-0
// tile a camera's Gaussian pyramid needs (each pixel's entry = that camera's map).  Per job the
// builder finds the cameras (<= 4 "slots") and their even-aligned luma boxes, and encodes each
// pixel as a 4-byte box-relative LDS byte offset + fractions + slot; jobs that do not
// fit (> 4 cameras, a box > 256 px, or LDS above kTileLdsBytes) become "wide" with 8-byte entries.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <cstdlib>
#include <thread>
#include <vector>

#include "host_common.hpp"
#include "kernels.hpp"

namespace octvr {

TiledLutBuild build_tiled_lut(const std::vector<TileJob>& jobs, const EntryFn& entry, const std::vector<int>& in_w,
                              const std::vector<int>& in_h, int qpl) {
    const int n_jobs = (int)jobs.size();
    const int item_px = kTilePx * qpl;  // qpl 128x8 halves stacked vertically
    TiledLutBuild b;
    b.qpl = qpl;
    b.hdr.resize(n_jobs);
    b.slots.resize((size_t)n_jobs * kTileSlots);
    b.entries.assign((size_t)n_jobs * item_px, 0u);
    std::vector<uint8_t> is_wide(n_jobs, 0);
    std::vector<std::vector<CompositeEntry>> wide_raw(n_jobs);
    std::vector<std::vector<uint16_t>> grp_job(n_jobs);  // per job its staging groups, chunk-padded
    const int T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::atomic<int> any_tex{0};  // some staged item holds texture-convention entries (b.tex)
    auto work = [&](int tid) {
        struct Px {
            int slot, x0, y0, fxy, mask, nogain;
        };
        std::vector<Px> px(item_px);
        std::vector<CompositeEntry> raw(item_px);
        for (int t = tid; t < n_jobs; t += T) {
            const TileJob& J = jobs[t];
            int cams[8], ns = 0;
            int minx[8], maxx[8], miny[8], maxy[8];
            bool wide = false, item_tex = false;
            for (int k = 0; k < item_px; k++) {
                // half h = k / kTilePx holds rows 8 h .. 8 h + 7; inside it quad-major (lane = quad)
                const int h = k / kTilePx, q = (k % kTilePx) >> 2, p = k & 3;
                const int x = J.tx * kTileW + (q & 63) * 2 + (p & 1);
                const int y = J.ty * kTileH * qpl + h * kTileH + (q >> 6) * 2 + (p >> 1);
                const CompositeEntry e = entry(t, x, y);
                raw[k] = e;
                px[k].mask = 0;
                if (!(e.code & 0x8000u)) continue;
                const int cam = (int)((e.code >> 10) & 31u);
                const int sx = (int)(int16_t)(e.xy & 0xFFFFu), sy = (int)(int16_t)(e.xy >> 16);
                const int iw = in_w[cam], ih = in_h[cam];
                int mask, fxy;
                if (e.code & kCodeTex) {
                    // texture-convention entry (make_entry_tex): a cell whose taps the clamp moves (on the
                    // image's border) takes the gather path; an interior one reads its four taps from the
                    // staged box like any other, with the 8-bit fractions in a 16-bit code
                    if (sx < 0 || sy < 0 || sx + 1 >= iw || sy + 1 >= ih) {
                        wide = true;
                        continue;
                    }
                    mask = 15;
                    fxy = (int)((e.code & 255u) | ((e.code >> 17) & 255u) << 8);
                    item_tex = true;
                } else {
                    const TapCell tc = tap_cell(e.xy, iw, ih);
                    mask = ((tc.ix0 && tc.iy0) ? 1 : 0) | ((tc.ix1 && tc.iy0) ? 2 : 0) | ((tc.ix0 && tc.iy1) ? 4 : 0) |
                           ((tc.ix1 && tc.iy1) ? 8 : 0);
                    if (!mask) continue;  // every tap outside: black
                    // a cell straddling the image's left or top edge (only in morphed / external LUTs):
                    // the staged boxes start inside the image, so the tile takes the gather path
                    if (sx < 0 || sy < 0) {
                        wide = true;
                        continue;
                    }
                    fxy = (int)(e.code & 1023u);
                }
                // here sx < iw and sy < ih; the +1 taps may sit on the zero column / row just past
                // the image, which the box then includes
                const int x0 = sx, y0 = sy, x1 = x0 + 1, y1 = y0 + 1;
                int sl = -1;
                for (int j = 0; j < ns; j++)
                    if (cams[j] == cam) sl = j;
                if (sl < 0) {
                    if (ns == 8) {
                        wide = true;
                        continue;
                    }
                    sl = ns++;
                    cams[sl] = cam;
                    minx[sl] = miny[sl] = INT32_MAX;
                    maxx[sl] = maxy[sl] = -1;
                }
                minx[sl] = std::min(minx[sl], x0);
                maxx[sl] = std::max(maxx[sl], x1);
                miny[sl] = std::min(miny[sl], y0);
                maxy[sl] = std::max(maxy[sl], y1);
                px[k] = Px{sl, x0, y0, fxy, mask, (e.code & kCodeNoGain) ? 1 : 0};
            }
            if (ns > kTileSlots) wide = true;
            TileSlot ts[kTileSlots] = {};
            int bws[kTileSlots] = {}, bhs[kTileSlots] = {};
            uint32_t stride = 0;
            for (int j = 0; j < ns && !wide; j++) {
                if (in_w[cams[j]] % 8) {  // dword staging of boxes needs 8-aligned box columns inside the image
                    wide = true;
                    break;
                }
                const int bx0 = minx[j] & ~7, by0 = miny[j] & ~1;
                const int bx1 = (maxx[j] + 1 + 7) & ~7, by1 = (maxy[j] + 1 + 1) & ~1;
                bws[j] = bx1 - bx0;
                bhs[j] = by1 - by0;
                if (bws[j] > 256 || bhs[j] > 256) {
                    wide = true;
                    break;
                }
                ts[j].cam = (uint16_t)cams[j];
                ts[j].bw = (uint16_t)bws[j];
                ts[j].bh = (uint16_t)bhs[j];
                ts[j].bx0 = (uint16_t)bx0;
                ts[j].by0 = (uint16_t)by0;
                stride = std::max<uint32_t>(stride, (uint32_t)bws[j]);
            }
            // Staged groups: per slot and box row, the 8-pixel groups from the row's leftmost to its
            // rightmost tap (row spans inside the box; the box keeps the LDS layout, so the entries'
            // tap offsets are unchanged, but the box's corners no tap reads are not staged)
            std::vector<uint16_t>& G = grp_job[t];
            G.clear();
            uint32_t chunks = 0, groups = 0;
            if (!wide) {
                std::vector<int> g_lo[kTileSlots], g_hi[kTileSlots];
                for (int j = 0; j < ns; j++) {
                    g_lo[j].assign(bhs[j], INT32_MAX);
                    g_hi[j].assign(bhs[j], -1);
                }
                for (int k = 0; k < item_px; k++) {
                    if (!px[k].mask) continue;
                    const int j = px[k].slot;
                    const int r = px[k].y0 - ts[j].by0, ga = (px[k].x0 - ts[j].bx0) >> 3, gb = (px[k].x0 + 1 - ts[j].bx0) >> 3;
                    for (int rr = r; rr <= r + 1; rr++) {
                        g_lo[j][rr] = std::min(g_lo[j][rr], ga);
                        g_hi[j][rr] = std::max(g_hi[j][rr], gb);
                    }
                }
                for (int j = 0; j < ns; j++) {
                    ts[j].chunk0 = (uint16_t)chunks;
                    uint32_t n = 0;
                    for (int r = 0; r < bhs[j]; r++)
                        for (int g = g_lo[j][r]; g <= g_hi[j][r]; g++, n++)
                            G.push_back((uint16_t)(kGroupValid | (uint32_t)g << 8 | (uint32_t)r));
                    const uint32_t c = (n + 63) / 64;
                    G.resize((size_t)(chunks + c) * 64, 0);  // the slot's last chunk padded with invalid groups
                    chunks += c;
                    groups += n;
                }
                // every tap of every pixel lies in a staged group of its slot (what the kernel reads from
                // LDS is exactly what staging wrote): checked here, once per rig
                std::vector<uint32_t> staged[kTileSlots];
                for (int j = 0; j < ns; j++) staged[j].assign(bhs[j], 0u);
                for (int j = 0; j < ns; j++) {
                    const uint32_t c_end = j + 1 < ns ? ts[j + 1].chunk0 : chunks;
                    for (uint32_t c = ts[j].chunk0; c < c_end; c++)
                        for (int i = 0; i < 64; i++) {
                            const uint16_t g = G[(size_t)c * 64 + i];
                            if (g & kGroupValid) staged[j][g & 255] |= 1u << ((g >> 8) & 31);
                        }
                }
                for (int k = 0; k < item_px; k++) {
                    if (!px[k].mask) continue;
                    const int j = px[k].slot, r = px[k].y0 - ts[j].by0;
                    const int ga = (px[k].x0 - ts[j].bx0) >> 3, gb = (px[k].x0 + 1 - ts[j].bx0) >> 3;
                    const uint32_t need = (1u << ga) | (1u << gb);
                    REQUIRE((staged[j][r] & need) == need && (staged[j][r + 1] & need) == need,
                            "tiled LUT: a tap outside the staged groups (internal error)");
                }
            }
            // Row stride of the staged boxes: the widest box, padded by 0-28 dwords to the value whose tap
            // reads conflict least in the LDS banks.  A tap read is a ds_read_b32 per dword (bank (a/4) mod 32,
            // lanes 0-31 and 32-63 one group each, MI355X_MICROARCH.md §LDS); a group's 32 lanes are 32 quads
            // of one quad row, whose taps lie on a curved strip across one or two box rows, so rows r and
            // r + 1 collide when the stride aliases the strip's spread onto the same banks.
            if (!wide && ns > 0) {
                uint32_t bh_sum = 0;
                for (int j = 0; j < ns; j++) bh_sum += (uint32_t)bhs[j];
                uint32_t lo[kTileSlots];
                auto cycles = [&](uint32_t S) {
                    uint32_t base = kTileZeroDwords;
                    for (int j = 0; j < ns; j++) {
                        lo[j] = base;
                        base += S * (uint32_t)bhs[j];
                    }
                    uint64_t cyc = 0;
                    uint32_t a[32];
                    for (int h = 0; h < qpl; h++)
                        for (int q0 = 0; q0 < 256; q0 += 32)
                            for (int p = 0; p < 4; p++) {
                                for (int l = 0; l < 32; l++) {
                                    const Px& x = px[(size_t)h * kTilePx + (size_t)(q0 + l) * 4 + p];
                                    const TileSlot& sl = ts[x.slot];
                                    a[l] = x.mask ? lo[x.slot] + (uint32_t)(x.y0 - sl.by0) * S + (uint32_t)(x.x0 - sl.bx0) : 0u;
                                }
                                for (int r = 0; r < 2; r++)
                                    for (int c = 0; c < 2; c++) {
                                        uint8_t cnt[32] = {};
                                        uint32_t seen[32][4];
                                        int mx = 1;
                                        for (int l = 0; l < 32; l++) {
                                            const uint32_t d = a[l] + (uint32_t)r * S + (uint32_t)c, bk = d & 31u;
                                            bool dup = false;
                                            for (int k = 0; k < std::min<int>(cnt[bk], 4); k++) dup |= seen[bk][k] == d;
                                            if (dup) continue;
                                            if (cnt[bk] < 4) seen[bk][cnt[bk]] = d;
                                            mx = std::max(mx, (int)++cnt[bk]);
                                        }
                                        cyc += (uint64_t)mx;
                                    }
                            }
                    return cyc;
                };
                uint32_t best = stride;
                uint64_t best_cyc = UINT64_MAX;
                for (uint32_t pad = 0; pad <= kStridePadMax; pad += kStageAlignDwords) {
                    const uint32_t S = stride + pad;
                    if ((kTileZeroDwords + S * bh_sum) * 4 > (uint32_t)kTileLdsBytes && pad > 0) break;
                    const uint64_t c = cycles(S);
                    if (c < best_cyc) {
                        best_cyc = c;
                        best = S;
                    }
                }
                stride = best;
            }
            uint32_t lds = kTileZeroDwords;
            for (int j = 0; j < ns && !wide; j++) {
                ts[j].lds = (uint16_t)std::min<uint32_t>(lds, 65535u);
                lds += stride * (uint32_t)bhs[j];
            }
            for (int j = ns; j < kTileSlots; j++) ts[j].chunk0 = (uint16_t)std::min<uint32_t>(chunks, 255u);
            if (chunks > 255) wide = true;
            if (lds * 4 > (uint32_t)kTileLdsBytes) wide = true;
            if (wide) {
                is_wide[t] = 1;
                wide_raw[t] = raw;
                G.clear();
                continue;
            }
            if (item_tex) any_tex = 1;
            b.hdr[t] = TileHdr{(uint32_t)J.tx | ((uint32_t)J.ty << 16),
                               (uint32_t)ns | (chunks << 8) | ((uint32_t)J.cam << 16),
                               2 * groups, stride};
            for (int j = 0; j < kTileSlots; j++) b.slots[(size_t)t * kTileSlots + j] = ts[j];
            uint32_t* out = b.entries.data() + (size_t)t * item_px;
            for (int k = 0; k < item_px; k++) {
                if (!px[k].mask) continue;  // black
                const TileSlot& sl = ts[px[k].slot];
                const uint32_t off = sl.lds + (uint32_t)(px[k].y0 - sl.by0) * stride + (uint32_t)(px[k].x0 - sl.bx0);
                out[k] = item_tex ? tiled_entry_tex(off * 4u, (uint32_t)px[k].fxy, (uint32_t)px[k].slot, px[k].nogain != 0)
                                  : tiled_entry(off * 4u, (uint32_t)px[k].fxy, (uint32_t)px[k].slot, px[k].nogain != 0);
            }
        }
    };
    run_threads((size_t)T, [&](size_t i) { work((int)i); });
    b.tex = any_tex.load();
    // staged items: the non-wide jobs in job order, compacted in place; wide jobs in job order
    int n_items = 0;
    for (int t = 0; t < n_jobs; t++) {
        if (is_wide[t]) {  // one 128x8 wide tile per half
            const TileJob& J = jobs[t];
            for (int h = 0; h < qpl; h++) {
                b.wide_tiles.push_back((uint32_t)J.tx | ((uint32_t)(J.ty * qpl + h) << 16));
                // the half's quarters as half 0's bits: results at bits 8-11, G0 at bits 12-15
                const uint32_t rq = (J.flags >> (4 * h)) & 15u, gq = (J.flags >> (8 + 4 * h)) & 15u;
                b.wide_cams.push_back((uint16_t)(J.cam | rq << 8 | gq << 12));
                b.wide.insert(b.wide.end(), wide_raw[t].begin() + (size_t)h * kTilePx,
                              wide_raw[t].begin() + (size_t)(h + 1) * kTilePx);
            }
            continue;
        }
        if (n_items != t) {
            b.hdr[n_items] = b.hdr[t];
            std::copy(b.slots.begin() + (size_t)t * kTileSlots, b.slots.begin() + (size_t)(t + 1) * kTileSlots,
                      b.slots.begin() + (size_t)n_items * kTileSlots);
            std::copy(b.entries.begin() + (size_t)t * item_px, b.entries.begin() + (size_t)(t + 1) * item_px,
                      b.entries.begin() + (size_t)n_items * item_px);
        }
        b.staged_bytes += 8.0 * b.hdr[n_items].stage_groups;  // 4 Y + 2 U + 2 V bytes per 4-pixel group
        b.item_flags.push_back((uint16_t)jobs[t].flags);
        // the item's first kGroupFirst chunks in its fixed grp0 block, the rest appended to grp1 (the
        // item's first overflow chunk in TileHdr::stride bits 9-31)
        {
            const std::vector<uint16_t>& G = grp_job[t];
            b.grp0.resize((size_t)(n_items + 1) * kGroupFirst * 64, 0);
            const size_t first = std::min<size_t>(G.size(), (size_t)kGroupFirst * 64);
            std::copy(G.begin(), G.begin() + first, b.grp0.begin() + (size_t)n_items * kGroupFirst * 64);
            const size_t ovf_chunk = b.grp1.size() / 64;
            REQUIRE(ovf_chunk < (1u << 23), "tiled LUT: staging group overflow table too large");
            b.hdr[n_items].stride |= (uint32_t)ovf_chunk << kStrideBits;
            b.grp1.insert(b.grp1.end(), G.begin() + first, G.end());
            std::vector<uint16_t>().swap(grp_job[t]);
        }
        n_items++;
    }
    b.n_items = n_items;
    b.n_wide = (int)b.wide_tiles.size();
    {  // unique source bytes the launch reads: the union over items of the staged groups (8 luma bytes per
       // group row, 4 U + 4 V bytes per group row pair), plus the wide tiles' tap cells
        const int nc = (int)in_w.size();
        std::vector<std::vector<uint8_t>> lum(nc), chr(nc);
        std::vector<int> cw(nc);
        for (int c = 0; c < nc; c++) {
            cw[c] = (in_w[c] + 7) / 8;
            lum[c].assign((size_t)cw[c] * in_h[c], 0);
            chr[c].assign((size_t)cw[c] * ((in_h[c] + 1) / 2), 0);
        }
        auto mark = [&](int c, int x, int y) {
            if (c < 0 || c >= nc || x < 0 || y < 0 || x >= in_w[c] || y >= in_h[c]) return;
            lum[c][(size_t)y * cw[c] + x / 8] = 1;
            chr[c][(size_t)(y / 2) * cw[c] + x / 8] = 1;
        };
        for (int t = 0; t < n_items; t++) {
            const int ns = (int)(b.hdr[t].nslots & 0xFFu), nch = (int)((b.hdr[t].nslots >> 8) & 0xFFu);
            for (int c = 0; c < nch; c++) {
                int j = 0;
                while (j + 1 < ns && c >= (int)b.slots[(size_t)t * kTileSlots + j + 1].chunk0) j++;
                const TileSlot& sl = b.slots[(size_t)t * kTileSlots + j];
                const uint16_t* g = c < kGroupFirst ? b.grp0.data() + ((size_t)t * kGroupFirst + c) * 64
                                                     : b.grp1.data() + ((size_t)(b.hdr[t].stride >> kStrideBits) + c - kGroupFirst) * 64;
                for (int i = 0; i < 64; i++)
                    if (g[i] & kGroupValid) mark(sl.cam, sl.bx0 + 8 * ((g[i] >> 8) & 31), sl.by0 + (g[i] & 255));
            }
        }
        for (const CompositeEntry& e : b.wide) {
            if (!(e.code & 0x8000u)) continue;
            const int c = (int)((e.code >> 10) & 31u);
            const int sx = (int)(int16_t)(e.xy & 0xFFFFu), sy = (int)(int16_t)(e.xy >> 16);
            for (int k = 0; k < 4; k++) mark(c, sx + (k & 1), sy + (k >> 1));
        }
        double groups = 0, pairs = 0;
        for (int c = 0; c < nc; c++) {
            for (uint8_t x : lum[c]) groups += x;
            for (uint8_t x : chr[c]) pairs += x;
        }
        b.source_bytes = groups * 8 + pairs * 8;
    }
    {  // XCD bands of equal item counts over the staged items (kernels.hpp kStitchBands)
        std::vector<double> cum(n_items + 1, 0.0);
        for (int t = 0; t < n_items; t++) cum[t + 1] = cum[t] + 1.0;
        b.bands.assign(kStitchBands + 1, n_items);
        b.bands[0] = 0;
        int t = 0;
        for (int g = 1; g < kStitchBands; g++) {
            const double goal = cum[n_items] * g / kStitchBands;
            while (t < n_items && cum[t] < goal) t++;
            b.bands[g] = std::max(t, b.bands[g - 1]);
        }
    }
    {  // build statistics (mapper info): how the staging work is distributed over items and bands
        const int edges[] = {0, 1, 2, 3, 4, 6, 8, 12, 16, 32, 256};
        const int n_bins = (int)(sizeof(edges) / sizeof(edges[0])) - 1;
        std::vector<long> hist(n_bins, 0), lds_hist(7, 0);
        std::vector<long> band_chunks(kStitchBands, 0);
        for (int t = 0; t < n_items; t++) {
            const int ch = (int)((b.hdr[t].nslots >> 8) & 0xFFu);
            int k = 0;
            while (k + 1 < n_bins && ch >= edges[k + 1]) k++;
            hist[k]++;
            uint32_t lds = kTileZeroDwords;
            for (int j = 0; j < (int)(b.hdr[t].nslots & 0xFFu); j++)
                lds += (b.hdr[t].stride & ((1u << kStrideBits) - 1)) * b.slots[(size_t)t * kTileSlots + j].bh;
            const uint32_t kb = lds * 4u / 1024u;  // 0-1, 1-2, 2-4, 4-8, 8-16, 16-24, >24 KiB
            lds_hist[kb < 1 ? 0 : kb < 2 ? 1 : kb < 4 ? 2 : kb < 8 ? 3 : kb < 16 ? 4 : kb < 24 ? 5 : 6]++;
            for (int g = 0; g < kStitchBands; g++)
                if (t >= b.bands[g] && t < b.bands[g + 1]) band_chunks[g] += ch;
        }
        std::string s = "\"items_by_chunks\": {";
        for (int k = 0; k < n_bins; k++)
            s += (k ? ", \"" : "\"") + std::to_string(edges[k]) + "\": " + std::to_string(hist[k]);
        s += "}, \"items_by_lds_kib\": [";
        for (int k = 0; k < 7; k++) s += (k ? ", " : "") + std::to_string(lds_hist[k]);
        s += "], \"band_chunks\": [";
        for (int g = 0; g < kStitchBands; g++) s += (g ? ", " : "") + std::to_string(band_chunks[g]);
        s += "]";
        b.stats = s;
    }
    b.hdr.resize(std::max(n_items, 1));
    b.grp0.resize((size_t)std::max(n_items, 1) * kGroupFirst * 64, 0);
    if (b.grp1.empty()) b.grp1.assign(64, 0);
    b.slots.resize((size_t)std::max(n_items, 1) * kTileSlots);
    b.entries.resize((size_t)std::max(n_items, 1) * item_px);
    if (b.wide.empty()) {
        b.wide.push_back(CompositeEntry{0, 0});
        b.wide_tiles.push_back(0u);
        b.wide_cams.push_back(0);
    }
    return b;
}

void TiledLutDev::upload(const TiledLutBuild& b, bool want_e24) {
    // per staged item one 80-byte record: its TileHdr, then its kTileSlots TileSlots (lane q of the
    // metadata load reads 16-byte word q)
    static_assert(sizeof(TileHdr) == 16 && sizeof(TileSlot) == 16, "16-byte metadata words");
    std::vector<TileHdr> m(b.hdr.size() * kMetaWords);
    for (size_t t = 0; t < b.hdr.size(); t++) {
        m[t * kMetaWords] = b.hdr[t];
        // word 2 on the device: the slot of each staging chunk c < 4 (2 bits at 2c), as stage_slot's
        // search over the slots' first chunks would find it (stage_groups is host-side statistics)
        uint32_t map = 0;
        const int ns = (int)(b.hdr[t].nslots & 0xFFu);
        for (int c = 0; c < 4; c++) {
            int q = 0;
            for (int j = 1; j < kTileSlots; j++) q += (j < ns && c >= (int)b.slots[t * kTileSlots + j].chunk0) ? 1 : 0;
            map |= (uint32_t)q << (2 * c);
        }
        if (t < b.item_flags.size()) map |= (uint32_t)b.item_flags[t] << 8;  // RGBA mode: item_result_bit / item_g0_bit
        m[t * kMetaWords].stage_groups = map;
        std::memcpy(&m[t * kMetaWords + 1], &b.slots[t * kTileSlots], kTileSlots * sizeof(TileSlot));
    }
    meta.upload(m.data(), m.size());
    REQUIRE(b.grp0.size() * 2 < (size_t)1 << 31 && b.grp1.size() * 2 < (size_t)1 << 31, "staging group tables exceed 2 GiB");
    grp0.upload(b.grp0.data(), b.grp0.size());
    grp1.upload(b.grp1.data(), b.grp1.size());
    // the composite addresses the entries through a buffer resource with 32-bit offsets
    REQUIRE(b.entries.size() * sizeof(uint32_t) < (size_t)1 << 32, "tiled LUT entries exceed 4 GiB");
    // 24-bit entries (tiled_entry24) when asked for and no entry carries "no gain" (the default sampling
    // only; OCTVR_ENTRY32=1 keeps the 32-bit layout: measurement knob).  Asked for by the multi-band remap
    // (C3 +3.4 %); the no-blend composite keeps 32-bit entries (C2 -1.5 % with 24: the two more VALU per
    // pixel cost more than the quarter of the entry fetches saves there; round 6, `e24ab`)
    bool e24 = want_e24 && !b.tex && std::getenv("OCTVR_ENTRY32") == nullptr;
    for (size_t k = 0; e24 && k < b.entries.size(); k++) e24 = (b.entries[k] & kEntryNoGain) == 0u;
    if (e24) {
        REQUIRE(b.entries.size() % 4 == 0, "tiled entries: whole quads");
        std::vector<uint32_t> p(b.entries.size() / 4 * 3);
        for (size_t q = 0; q < b.entries.size() / 4; q++) {
            const uint32_t c0 = tiled_entry24(b.entries[4 * q]), c1 = tiled_entry24(b.entries[4 * q + 1]);
            const uint32_t c2 = tiled_entry24(b.entries[4 * q + 2]), c3 = tiled_entry24(b.entries[4 * q + 3]);
            p[3 * q] = c0 | c1 << 24;
            p[3 * q + 1] = c1 >> 8 | c2 << 16;
            p[3 * q + 2] = c2 >> 16 | c3 << 8;
        }
        entries.upload(p.data(), p.size());
    } else {
        entries.upload(b.entries.data(), b.entries.size());
    }
    wide.upload(b.wide.data(), b.wide.size());
    wide_tiles.upload(b.wide_tiles.data(), b.wide_tiles.size());
    wide_cams.upload(b.wide_cams.data(), b.wide_cams.size());
    bands.upload(b.bands.data(), b.bands.size());
    queue.alloc((size_t)(kStitchBands + 1) * kQueueStride);
    HIP_CHECK(hipMemset(queue.p, 0, queue.n * sizeof(uint32_t)));
    staged_bytes = b.staged_bytes;
    source_bytes = b.source_bytes;
    result_bytes = 0;
    g0_bytes = 0;
    constexpr double kSubPx = (double)kSubW * kTileH;
    for (size_t t = 0; t < b.item_flags.size(); t++) {
        const uint32_t f = b.item_flags[t];
        g0_bytes += 4.0 * kSubPx * __builtin_popcount(f & 0xFF00u);
        result_bytes += kSubPx * __builtin_popcount(f & 0xFFu);  // result pixels (bytes: x 1.5 or 4)
    }
    if (!b.item_flags.empty())
        for (uint16_t c : b.wide_cams) {
            g0_bytes += 4.0 * kSubPx * __builtin_popcount((uint32_t)c >> 12);
            result_bytes += kSubPx * __builtin_popcount(((uint32_t)c >> 8) & 15u);
        }
    if (b.item_flags.empty()) g0_bytes = 4.0 * kTilePx * ((double)b.n_items * b.qpl + b.n_wide);  // no flags: every half
    stats = b.stats;
    view = TiledLut{meta.p, entries.p, b.n_items, wide_tiles.p, wide.p, b.n_wide, wide_cams.p, bands.p, queue.p,
                    b.qpl, grp0.p, grp1.p, (uint32_t)b.grp1.size(), b.tex, e24 ? 1 : 0};
}

void SourceFootprint::init(const std::vector<int>& in_w, const std::vector<int>& in_h) {
    w = in_w;
    h = in_h;
    bits.assign(w.size(), {});
    for (size_t i = 0; i < w.size(); i++) bits[i].assign((size_t)row_pairs((int)i) * words((int)i), 0ull);
}

void SourceFootprint::mark_taps(const CompositeEntry& e) {
    if (!(e.code & 0x8000u)) return;
    const int cam = (int)((e.code >> 10) & 31u);
    if (cam >= (int)w.size()) return;
    const TapCell c = tap_cell(e.xy, w[cam], h[cam]);
    const bool all = (e.code & kCodeTex) != 0;  // texture convention: all four clamped taps are used
    if (all || (c.iy0 && c.ix0)) mark(cam, c.y0, c.x0 >> 3);
    if (all || (c.iy0 && c.ix1)) mark(cam, c.y0, c.x1 >> 3);
    if (all || (c.iy1 && c.ix0)) mark(cam, c.y1, c.x0 >> 3);
    if (all || (c.iy1 && c.ix1)) mark(cam, c.y1, c.x1 >> 3);
}

void SourceFootprint::merge(const SourceFootprint& o) {
    REQUIRE(o.w == w && o.h == h, "footprints of different input sizes");
    for (size_t i = 0; i < bits.size(); i++)
        for (size_t k = 0; k < bits[i].size(); k++) bits[i][k] |= o.bits[i][k];
}

double SourceFootprint::bytes() const {
    double n = 0;
    for (int i = 0; i < (int)w.size(); i++)
        for (int r = 0; r < row_pairs(i); r++)
            for (int g = 0; g < groups(i); g++) {
                if (!test(i, r, g)) continue;
                const int yb = std::min(8, w[i] - 8 * g), cb = std::max(0, std::min(4, w[i] / 2 - 4 * g));
                n += yb * (2 * r + 1 < h[i] ? 2 : 1) + 2 * cb;
            }
    return n;
}

void footprint_add_tiles(SourceFootprint& f, const TiledLutBuild& b) {
    for (int t = 0; t < b.n_items; t++) {
        const TileHdr& hd = b.hdr[t];
        const int ns = (int)(hd.nslots & 0xFFu), nch = (int)((hd.nslots >> 8) & 0xFFu);
        const TileSlot* ts = b.slots.data() + (size_t)t * kTileSlots;
        for (int c = 0; c < nch; c++) {
            int j = 0;  // the chunk's slot (slots own consecutive chunk ranges from chunk0)
            for (int k = 1; k < ns; k++)
                if (c >= (int)ts[k].chunk0) j = k;
            const uint16_t* G = c < kGroupFirst ? b.grp0.data() + ((size_t)t * kGroupFirst + c) * 64
                                                : b.grp1.data() + ((size_t)(hd.stride >> kStrideBits) + c - kGroupFirst) * 64;
            const int cam = ts[j].cam;
            for (int l = 0; l < 64; l++) {
                if (!(G[l] & kGroupValid)) continue;
                const int y = ts[j].by0 + (G[l] & 255), x = ts[j].bx0 + ((G[l] >> 8) & 31) * 8;
                if (y < f.h[cam] && x < f.w[cam]) f.mark(cam, y, x >> 3);  // else staged as black, unread
            }
        }
    }
    for (const CompositeEntry& e : b.wide) f.mark_taps(e);
}

}  // namespace octvr
