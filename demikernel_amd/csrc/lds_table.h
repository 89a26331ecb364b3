// lds_table.h — host builder of the LDS copy of the Active socket table (rx_common.h: minimal perfect hash). Host code
// only (no HIP calls), so the ASan + UBSan harness (tests/host_asan) links it too.
#pragma once

#include <algorithm>
#include <cstdint>
#include <vector>

#include "rx_common.h"

namespace dk {

// From the built open-addressing slots (so duplicates resolve exactly as there), the Active connections with
// local_ip == cfg_ip (the only ones a reference lookup can ask for). Buckets are placed largest first, each with the
// smallest displacement that puts all its keys on free slots. Returns false (no LDS table: lookups probe the global
// table) for no keys, more than kLtMaxKeys, keys whose 32-bit hashes collide (they can never be separated: checked up
// front on the sorted hashes, so such a table costs no displacement search), or no displacement below 2^20 for a
// bucket.
inline bool build_lds_table(const std::vector<uint32_t>& slots, uint32_t cap, uint32_t cfg_ip,
                            std::vector<uint32_t>& out, uint32_t& n_out, uint32_t& b_out) {
    struct Key {
        uint32_t h, rip, ports, fid;
    };
    std::vector<Key> keys;
    if (slots.size() < (size_t)cap * 4) return false;
    for (uint32_t i = 0; i < cap; i++) {
        const uint32_t* sl = &slots[(size_t)i * 4];
        if (sl[0] == 0 || (sl[0] >> 24) != DK_FLOW_TCP_ACTIVE || sl[1] != cfg_ip) continue;
        if (keys.size() >= kLtMaxKeys) return false;
        keys.push_back({flow_hash(DK_FLOW_TCP_ACTIVE, cfg_ip, sl[2], sl[3]), sl[2], sl[3], sl[0] & 0xFFFFFFu});
    }
    const uint32_t n = (uint32_t)keys.size();
    if (n == 0) return false;
    {
        std::vector<uint32_t> hs(n);
        for (uint32_t k = 0; k < n; k++) hs[k] = keys[k].h;
        std::sort(hs.begin(), hs.end());
        if (std::adjacent_find(hs.begin(), hs.end()) != hs.end()) return false;  // two keys, one hash
    }
    const uint32_t nb = (n + 3) / 4;
    std::vector<std::vector<uint32_t>> bucket(nb);
    for (uint32_t k = 0; k < n; k++) bucket[lt_bucket(keys[k].h, nb)].push_back(k);
    std::vector<uint32_t> order(nb);
    for (uint32_t b = 0; b < nb; b++) order[b] = b;
    std::stable_sort(order.begin(), order.end(),
                     [&](uint32_t a, uint32_t b) { return bucket[a].size() > bucket[b].size(); });
    std::vector<uint8_t> taken(n, 0);
    std::vector<uint32_t> disp(nb, 0), slot_of(n, 0), at;
    for (uint32_t b : order) {
        if (bucket[b].empty()) break;
        uint32_t d = 0;
        for (;; d++) {
            if (d >= (1u << 20)) return false;
            at.clear();
            bool ok = true;
            for (uint32_t k : bucket[b]) {
                const uint32_t sl = lt_slot(keys[k].h, d, n);
                if (taken[sl] || std::find(at.begin(), at.end(), sl) != at.end()) {
                    ok = false;
                    break;
                }
                at.push_back(sl);
            }
            if (ok) break;
        }
        disp[b] = d;
        for (size_t j = 0; j < at.size(); j++) {
            taken[at[j]] = 1;
            slot_of[bucket[b][j]] = at[j];
        }
    }
    out.assign(lt_words(n, nb), 0u);
    for (uint32_t k = 0; k < n; k++) {
        out[slot_of[k]] = keys[k].rip;
        out[n + slot_of[k]] = keys[k].ports;
        out[2 * n + slot_of[k]] = keys[k].fid;
    }
    std::copy(disp.begin(), disp.end(), out.begin() + 3 * n);
    n_out = n;
    b_out = nb;
    return true;
}

// The compact UDP bind table (rx_common.h) from the port table's kPortUdpLocal words (65,536, DK_FLOW_NONE where no
// bind): 2 (mask + 1) words, the seed that placed every bind, and the 128-byte lines of the port table the binds' words
// occupy (the host reads the compact table instead when that is more than it takes). Cuckoo insertion (a displaced
// word moves to its other bucket) with up to 500 displacements per bind, seeds 0..63. Returns false (local binds stay
// on the port table) for no binds, more than kUbMaxBinds, a flow id >= 0xFFFF, or no seed that places them all.
inline bool build_udp_table(const uint32_t* local, std::vector<uint32_t>& out, uint32_t& mask, uint32_t& seed,
                            uint32_t& direct_lines) {
    std::vector<uint32_t> keys;  // port | fid << 16
    direct_lines = 0;
    uint32_t last_line = ~0u;
    for (uint32_t port = 0; port < 65536; port++) {
        const uint32_t fid = local[port];
        if (fid == DK_FLOW_NONE) continue;
        if (fid >= 0xFFFFu || keys.size() >= kUbMaxBinds) return false;
        keys.push_back(port | fid << 16);
        if (port >> 5 != last_line) direct_lines++;
        last_line = port >> 5;
    }
    if (keys.empty()) return false;
    uint32_t nb = 16;
    while (nb < keys.size()) nb <<= 1;
    const uint32_t m = nb - 1;
    for (uint32_t sd = 0; sd < 64; sd++) {
        out.assign(2 * (size_t)nb, kUbEmpty);
        bool ok = true;
        for (size_t k = 0; k < keys.size() && ok; k++) {
            uint32_t e = keys[k], from = ~0u;  // from: the bucket e was displaced out of
            for (int kick = 0;; kick++) {
                const uint32_t h = ub_hash(e & 0xFFFFu, sd), b1 = h & m, b2 = (h >> 16) & m;
                bool placed = false;
                for (uint32_t b : {b1, b2})
                    for (uint32_t w = 0; w < 2 && !placed; w++)
                        if (out[2 * b + w] == kUbEmpty) {
                            out[2 * b + w] = e;
                            placed = true;
                        }
                if (placed) break;
                if (kick == 500) {
                    ok = false;
                    break;
                }
                const uint32_t b = from == b1 ? b2 : b1;  // not back into the bucket it just left
                std::swap(e, out[2 * b + (uint32_t)(kick & 1)]);
                from = b;
            }
        }
        if (ok) {
            mask = m;
            seed = sd;
            return true;
        }
    }
    return false;
}

}  // namespace dk
