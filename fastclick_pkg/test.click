// GPUIPCheckClassify in a FastClick graph (userlevel, no DPDK needed):
//   CLICKPATH=$PWD click test.click TRACE=trace.pcap
// Behind FromDPDKDevice the element takes FromDump's place unchanged.
require(package "gpu");
define($TRACE trace.pcap)

FromDump($TRACE, STOP true, BURST 32)
  -> gpu :: GPUIPCheckClassify(OFFSET 14, CHECKSUM true, N 4, LB_MODE hash, DETAILS true,
                               BATCH 8192, TIMER 100);
gpu[0] -> c0 :: Counter -> Discard;
gpu[1] -> c1 :: Counter -> Discard;
gpu[2] -> c2 :: Counter -> Discard;
gpu[3] -> c3 :: Counter -> Discard;
gpu[4] -> bad :: Counter -> Discard;    // packets CheckIPHeader would drop

DriverManager(wait, wait 10ms,
              print gpu.count, print gpu.drops, print gpu.drop_details,
              print c0.count, print c1.count, print c2.count, print c3.count, print bad.count)
