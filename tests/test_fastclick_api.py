"""The FastClick package element (fastclick_pkg/) against the reference's API.

This container has no FastClick install and the pipeline does not run the
reference's configure (which generates click/config.h), so the package is not
compiled here. What can be checked is that every FastClick declaration the
element and its ClickPolicy use exists in the reference headers with the
signature the element relies on. Reads /root/reference (CPU only; skipped
where the reference tree is absent, e.g. on the GPU box).
"""
import os
import re

import pytest

REF = "/root/reference/include/click"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# (header, pattern of the declaration the package relies on, what uses it)
API = [
    ("batchelement.hh", r"class BatchElement : public Element", "GPUIPCheckClassify base class"),
    ("batchelement.hh", r"inline void checked_output_push_batch\(int port, PacketBatch\* batch\)", "output runs"),
    ("element.hh", r"enum batch_mode \{BATCH_MODE_NO, BATCH_MODE_IFPOSSIBLE, BATCH_MODE_NEEDED", "in_batch_mode"),
    ("element.hh", r"virtual void run_timer\(Timer \*timer\);", "TIMER flush"),
    ("element.hh", r"Bitvector get_passing_threads\(bool touching = false\);", "per-thread cores"),
    ("element.hh", r"int home_thread_id\(\) const;", "fallback thread"),
    ("element.hh", r"void add_read_handler\(const String &name, ReadHandlerCallback read_callback, int user_data",
     "handlers"),
    ("element.hh", r"static const char PUSH\[\];", "processing()"),
    ("packet.hh", r"inline const unsigned char \*data\(\) const;", "ClickPolicy::data"),
    ("packet.hh", r"inline uint32_t length\(\) const;", "ClickPolicy::length"),
    ("packet.hh", r"inline Packet \*next\(\) const;", "ClickPolicy::next"),
    ("packet.hh", r"inline void set_next\(Packet \*p\);", "ClickPolicy::set_next"),
    ("packet.hh", r"inline void kill\(\);", "ClickPolicy::kill"),
    ("packet.hh", r"void set_anno_u8\(int i, uint8_t x\)", "annotations"),
    ("packet.hh", r"void set_anno_u16\(int i, uint16_t x\)", "annotations"),
    ("packet.hh", r"void set_anno_u32\(int i, uint32_t x\)", "annotations"),
    ("packet.hh", r"inline void set_network_header\(const unsigned char \*p, uint32_t len\);", "set_headers"),
    ("packet.hh", r"void take\(uint32_t len\);", "ClickPolicy::take"),
    ("packet.hh", r"void pull\(uint32_t len\);", "ClickPolicy::pull"),
    ("packet.hh", r"inline WritablePacket \*uniqueify\(\)", "header rewrites"),
    ("packet.hh", r"anno_size = 48", "FLOWID_ANNO bound"),
    ("packetbatch.hh", r"inline static PacketBatch\* make_from_simple_list\(Packet\* head, Packet\* tail, unsigned int size\)",
     "ClickPolicy::make_batch"),
    ("packetbatch.hh", r"#define MAX_BATCH_SIZE 8192", "RxCore::kMaxBatch"),
    ("packet_anno.hh", r"#define DST_IP_ANNO_OFFSET\s+0", "kDstIp"),
    ("packet_anno.hh", r"#define IP6_NXT_ANNO_OFFSET\s+16", "kIp6Nxt"),
    ("packet_anno.hh", r"#define PAINT_ANNO_OFFSET\s+17", "kPaint"),
    ("packet_anno.hh", r"#define VLAN_TCI_ANNO_OFFSET\s+20", "kVlanTci"),
    ("packet_anno.hh", r"#define AGGREGATE_ANNO_OFFSET\s+20", "kAggregate"),
    ("timer.hh", r"Timer\(Element \*element\);", "per-thread Timer"),
    ("timer.hh", r"void schedule_after\(const Timestamp &delta\);", "arm()"),
    ("timer.hh", r"inline bool scheduled\(\) const", "arm()"),
    ("timer.hh", r"inline const Timestamp &expiry_steady\(\) const", "arm(): an earlier deadline moves the timer up"),
    ("element.hh", r"inline int noutputs\(\) const", "ERROR_OUTPUT check, Emit::noutputs"),
    ("timer.hh", r"void move_thread\(int tid\);", "per-thread Timer"),
    ("timer.hh", r"void initialize\(Element \*owner, bool quiet = false\);", "per-thread Timer"),
    ("timer.hh", r"inline void clear\(\)", "cleanup"),
    ("timestamp.hh", r"static inline Timestamp now_steady\(\);", "ClickPolicy::now_ns"),
    ("timestamp.hh", r"static inline Timestamp make_nsec\(value_type nsec\)", "arm()"),
    ("timestamp.hh", r"inline value_type nsecval\(\) const", "ClickPolicy::now_ns"),
    ("sync.hh", r"class per_thread", "per-thread state"),
    ("sync.hh", r"inline T& get_value_for_thread\(int thread_id\) const", "per-thread state"),
    ("sync.hh", r"inline unsigned weight\(\) const", "handlers, cleanup"),
    ("sync.hh", r"inline T\* operator->\(\) const", "per-thread state"),
    ("glue.hh", r"click_current_cpu_id\(\)", "lazy per-thread core"),
]


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference headers not present")
@pytest.mark.parametrize("header,pattern,use", API)
def test_reference_declares(header, pattern, use):
    src = open(os.path.join(REF, header)).read()
    assert re.search(pattern, src), f"{header}: no `{pattern}` ({use})"


def test_package_uses_only_checked_api():
    """Every Packet/PacketBatch/Timer member the package calls appears in the
    list above (so a new use cannot slip past this check)."""
    src = open(os.path.join(ROOT, "fastclick_pkg", "gpuipcheckclassify.hh")).read() + \
        open(os.path.join(ROOT, "fastclick_pkg", "gpuipcheckclassify.cc")).read()
    used = set(re.findall(r"(?:->|\.)([a-z_][a-z_0-9]*)\(", src))
    checked = set()
    for _, pat, _ in API:
        checked |= set(re.findall(r"([a-z_][a-z_0-9]*)\\\(", pat))
    # members of the element's own state/core and of std types are not FastClick API
    own = {"push_list", "push_one", "run_timer", "configure", "initialize", "counters", "nports", "details",
           "error", "timer_us", "idle", "staged", "due_ns", "get", "c_str", "push_back", "clear", "size",
           "first", "get_passing_threads", "error", "name", "checked_output_push_batch", "make_state",
           "read_handler", "empty", "error_output", "flow_timeouts", "maint_due_ns"}
    missing = used - checked - own
    assert not missing, f"unchecked FastClick calls: {sorted(missing)}"
