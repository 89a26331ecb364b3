// dk_tcp_oracle.cpp — TEST INFRASTRUCTURE ONLY (loaded by oracle/oracle.py; used by tests/ as the checker of
// dk_tcp_rx_process, never by the product): a CPU restatement of the reference's established-state TCP receive
// processing, segment by segment, per connection. Paths relative to /root/reference/src/rust/inetstack/protocols/
// layer4/tcp/:
//   ControlBlock::poll                     established/ctrlblk.rs:350-398 (stops after RST / FIN: later segments wait)
//   process_packet                         :403-440
//   check_segment_in_window                :447-567
//   check_rst / check_syn                  :570-604
//   process_ack                            :607-650 (the ack_num <= SND.NXT test; the sender side is out of scope)
//   process_data                           :652-695
//   get_receive_window_size                :786-789
//   store_out_of_order_fin / _segment      :836-941 (VecDeque; MAX_OUT_OF_ORDER_SIZE_FRAMES = 16, :53)
//   receive_data                           :951-1001
//   process_remote_close                   :1003-1024
//   Receiver::push                         :131-136 (RCV.NXT += buffer length)
//   SeqNumber < <= >=                      sequence_number.rs:76-101
//   DemiBuffer adjust / trim               runtime/memory/demibuffer.rs:515-590
// The out-of-order store is a std::deque like the reference's VecDeque (the GPU walker keeps fixed arrays).
#include <cstdint>
#include <deque>
#include <utility>
#include <vector>

#include "../include/dk_tcp.h"

namespace {

bool slt(uint32_t a, uint32_t b) { return (int32_t)(a - b) < 0; }
bool sle(uint32_t a, uint32_t b) { return (int32_t)(a - b) <= 0; }
bool sge(uint32_t a, uint32_t b) { return (int32_t)(a - b) >= 0; }

struct Buf {  // a DemiBuffer view
    uint32_t ref, off, len;
    void adjust(uint32_t k) {
        off += k;
        len -= k;
    }
    void trim(uint32_t k) { len -= k; }
    dk_tcp_view view() const { return dk_tcp_view{ref, off, len}; }
};

struct Conn {
    dk_tcp_conn* s;
    std::deque<std::pair<uint32_t, Buf>> ooo;  // receive_out_of_order_frames
    std::vector<dk_tcp_view> pushed;           // the receive queue, in push order
    void push(const Buf& b) {                  // Receiver::push
        pushed.push_back(b.view());
        s->receive_next += b.len;
    }
};

// store_out_of_order_segment (ctrlblk.rs:844-941).
uint32_t store_out_of_order_segment(Conn& c, uint32_t new_start, uint32_t new_end, Buf buf) {
    size_t action_index = c.ooo.size();
    bool another_pass = true;
    while (another_pass) {
        another_pass = false;
        action_index = c.ooo.size();
        for (size_t index = 0; index < c.ooo.size(); index++) {
            const uint32_t stored_start = c.ooo[index].first;
            const uint32_t stored_len = c.ooo[index].second.len;
            const uint32_t stored_end = stored_start + (stored_len - 1);
            if (slt(new_start, stored_start)) {
                if (slt(new_end, stored_start)) {  // entirely before
                    action_index = index;
                    break;
                }
                if (slt(stored_end, new_end)) {  // encompasses the stored segment: drop it, scan again
                    another_pass = true;
                    action_index = index;
                    break;
                }
                const uint32_t excess = (new_end - stored_start) + 1;  // front overlap: trim the new segment's end
                new_end = new_end - excess;
                buf.trim(excess);
                break;  // (action_index stays at the end of the store, as in the reference)
            }
            if (sle(new_end, stored_end)) return DK_TCP_STORE_DUP;  // complete duplicate
            if (slt(stored_end, new_start)) continue;                // entirely after
            const uint32_t duplicate = stored_end - new_start;       // end overlap (one byte short, as the reference)
            new_start = new_start + duplicate;
            buf.adjust(duplicate);
        }
        if (another_pass) c.ooo.erase(c.ooo.begin() + (std::ptrdiff_t)action_index);
    }
    c.ooo.insert(c.ooo.begin() + (std::ptrdiff_t)action_index, {new_start, buf});
    while (c.ooo.size() > DK_TCP_OOO_MAX) c.ooo.pop_back();
    return DK_TCP_STORED;
}

// receive_data (ctrlblk.rs:951-1001): true if a stored FIN is now in order.
bool receive_data(Conn& c, Buf buf) {
    uint32_t recv_next = c.s->receive_next + buf.len;
    c.push(buf);
    while (!c.ooo.empty()) {
        if (c.ooo.front().first != recv_next) break;
        const Buf t = c.ooo.front().second;
        c.ooo.pop_front();
        recv_next = recv_next + t.len;
        c.push(t);
    }
    return c.s->fin_pending && c.s->fin_seq == recv_next;
}

// process_packet (ctrlblk.rs:403-440) for one segment: returns the enum dk_tcp_action.
uint32_t process_packet(Conn& c, uint32_t seq, uint32_t ack_num, uint32_t flags, Buf data, dk_tcp_view& view) {
    dk_tcp_conn& s = *c.s;
    bool syn = flags & 0x02u, fin = flags & 0x01u;
    const bool rst = flags & 0x04u, ack = flags & 0x10u;
    uint32_t seg_start = seq, seg_end = seq, seg_len = data.len;
    view = data.view();

    // check_segment_in_window
    if (syn) seg_len += 1;
    if (fin) seg_len += 1;
    if (seg_len > 0) seg_end = seg_start + (seg_len - 1);
    const uint32_t receive_next = s.receive_next;
    const uint32_t window = s.buffer_size - (receive_next - s.reader_next);  // get_receive_window_size
    const uint32_t after_receive_window = receive_next + window;
    if (seg_start != receive_next) {
        if (slt(seg_start, receive_next)) {
            if (slt(seg_end, receive_next)) return DK_TCP_DUPLICATE;
            uint32_t duplicate = receive_next - seg_start;
            seg_start = seg_start + duplicate;
            seg_len -= duplicate;
            if (syn) {
                syn = false;
                duplicate -= 1;
            }
            data.adjust(duplicate);
        } else if (sge(seg_start, after_receive_window)) {
            return DK_TCP_OUT_OF_WINDOW;
        }
    }
    if (seg_len > 0 && sge(seg_end, after_receive_window)) {
        uint32_t excess = (seg_end - after_receive_window) + 1;
        seg_end = seg_end - excess;
        seg_len -= excess;
        if (fin) {
            fin = false;
            excess -= 1;
        }
        data.trim(excess);
    }
    view = data.view();

    if (rst) {  // check_rst: ECONNRESET ends the poll loop
        s.state = DK_TCP_CLOSED;
        return DK_TCP_RST;
    }
    if (syn) return DK_TCP_SYN;                                  // check_syn
    if (!ack) return DK_TCP_NO_ACK;                              // process_ack
    if (!sle(ack_num, s.send_next)) return DK_TCP_ACK_UNSENT;

    uint32_t action = DK_TCP_NO_DATA;
    if (data.len > 0 || fin) {  // process_data
        if (seg_start != s.receive_next) {
            action = DK_TCP_STORED;
            if (seg_len > 0) {
                if (fin) {
                    seg_len -= 1;
                    s.fin_pending = 1;  // store_out_of_order_fin
                    s.fin_seq = seg_end;
                    seg_end = seg_end - 1;
                    fin = false;
                }
                if (seg_len > 0) action = store_out_of_order_segment(c, seg_start, seg_end, data);
            }
        } else {
            action = DK_TCP_DELIVERED;
            if (receive_data(c, data)) fin = true;
        }
    }
    if (fin) {  // process_remote_close
        c.push(Buf{DK_TCP_REF_EOF, 0, 0});
        s.receive_next = s.receive_next + 1;
        s.state = DK_TCP_CLOSED;
        return DK_TCP_FIN;
    }
    return action;
}

}  // namespace

// The batch, in the dk_tcp_rx_process output layout (include/dk_tcp.h).
extern "C" int dko_tcp_process(dk_tcp_conn* conns, uint32_t nconns, uint32_t n, const uint32_t* meta,
                               const uint32_t* flow_id, const uint32_t* seq, const uint32_t* ack,
                               const uint32_t* payload, uint8_t* action, dk_tcp_view* view, dk_tcp_view* deliv,
                               uint32_t* deliv_start, uint32_t* deliv_count) {
    std::vector<std::vector<uint32_t>> segs(nconns);
    for (uint32_t i = 0; i < n; i++) {
        action[i] = DK_TCP_SKIP;
        view[i] = dk_tcp_view{i, payload[i] & 0xFFFFu, payload[i] >> 16};
        if ((meta[i] & 0xFFu) != DK_V_OK_TCP) continue;
        const uint32_t f = flow_id[i];
        if (f < nconns && conns[f].state != DK_TCP_NONE) segs[f].push_back(i);
    }
    uint64_t before = 0;
    for (uint32_t c = 0; c < nconns; c++) {
        dk_tcp_conn& s = conns[c];
        deliv_start[c] = (uint32_t)(before + (uint64_t)DK_TCP_DELIV_EXTRA * c);
        Conn cc{&s, {}, {}};
        for (uint32_t k = 0; k < s.ooo_count && k < DK_TCP_OOO_MAX; k++)
            cc.ooo.push_back({s.ooo_start[k], Buf{s.ooo[k].ref, s.ooo[k].off, s.ooo[k].len}});
        for (uint32_t i : segs[c]) {
            if (s.state != DK_TCP_ESTABLISHED) {
                action[i] = DK_TCP_UNPROCESSED;
                continue;
            }
            const uint32_t p = payload[i];
            action[i] = (uint8_t)process_packet(cc, seq[i], ack[i], (meta[i] >> 16) & 0xFFu,
                                                Buf{i, p & 0xFFFFu, p >> 16}, view[i]);
        }
        s.ooo_count = (uint32_t)cc.ooo.size();
        for (uint32_t k = 0; k < DK_TCP_OOO_MAX; k++) {
            const bool live = k < cc.ooo.size();
            s.ooo_start[k] = live ? cc.ooo[k].first : 0u;
            s.ooo[k] = live ? cc.ooo[k].second.view() : dk_tcp_view{0, 0, 0};
        }
        for (size_t k = 0; k < cc.pushed.size(); k++) deliv[deliv_start[c] + k] = cc.pushed[k];
        deliv_count[c] = (uint32_t)cc.pushed.size();
        before += segs[c].size();
    }
    return 0;
}
