#!/usr/bin/env python3
"""Test-only click/config.h + click/config-userlevel.h for compile-checking
the FastClick package element without running the reference's configure.

autoconf's config.status turns every `#undef NAME` line of a config.h.in into
`#define NAME VALUE` (a feature the configure run found) or leaves it
commented out. This script does the same substitution with a fixed answer
set: the one a userlevel x86-64 Linux gcc build with batching, flows, IPv6
and user multithreading gives (the survey's configuration, SURVEY.md §8(c):
--enable-userlevel --enable-ip6 --enable-flow --disable-dynamic-linking
--disable-verbose-batch), with no DPDK/netmap/pcap. Everything not listed
stays undefined, as configure leaves an absent feature.

    python3 fastclick_pkg/gen_config.py REFERENCE_DIR OUT_DIR
        -> OUT_DIR/click/config.h, OUT_DIR/click/config-userlevel.h

Only tests use it (tests/test_fastclick_pkg.py): it produces headers for
`g++ -fsyntax-only`, never a FastClick build.
"""
from __future__ import annotations

import os
import re
import sys

# config.h.in (CLICK_VERSION from configure.in's AC_INIT([click], [2.1]))
CONFIG_H = {
    "CLICK_BYTE_ORDER": "CLICK_LITTLE_ENDIAN",
    "CLICK_VERSION": '"2.1"',
    "CLICK_VERSION_CODE": "CLICK_MAKE_VERSION_CODE(2,1,0)",
    "HAVE___BUILTIN_CTZ": "1", "HAVE___BUILTIN_CLZ": "1", "HAVE___BUILTIN_CLZL": "1",
    "HAVE___BUILTIN_CLZLL": "1", "HAVE___BUILTIN_FFS": "1", "HAVE___BUILTIN_FFSL": "1",
    "HAVE___BUILTIN_FFSLL": "1", "HAVE___BUILTIN_POPCOUNT": "1",
    "HAVE___IS_TRIVIALLY_COPYABLE": "1",
    "HAVE___SYNC_SYNCHRONIZE": "1",
    "HAVE_ADDRESSABLE_VA_LIST": "1",
    "HAVE_ARITHMETIC_RIGHT_SHIFT": "1",
    "HAVE_BATCH": "1",
    "HAVE_AUTO_BATCH": "1",
    "HAVE_CXX_CONSTEXPR": "1",
    "HAVE_CXX_RVALUE_REFERENCES": "1",
    "HAVE_CXX_STATIC_ASSERT": "1",
    "HAVE_CXX_TEMPLATE_ALIAS": "1",
    "HAVE_FLOW": "1",
    "HAVE_INDIFFERENT_ALIGNMENT": "1",
    "HAVE_INT64_TYPES": "1",
    "HAVE_IP6": "1",
    "HAVE_LONG_LONG": "1",
    "HAVE_STRUCT_TIMESPEC": "1",
    "HAVE_USER_TIMING": "1",
    "SIZEOF_INT": "4", "SIZEOF_LONG": "8", "SIZEOF_LONG_LONG": "8", "SIZEOF_SIZE_T": "8",
    "SIZEOF_STRUCT_TIMESPEC": "16", "SIZEOF_STRUCT_TIMEVAL": "16", "SIZEOF_PTRDIFF_T": "8",
    "SIZEOF_VOID_P": "8",
    "HAVE_SSE2": "1",
    "__MTCLICK__": "1",
}

# config-userlevel.h.in
CONFIG_USERLEVEL_H = {
    "HAVE___THREAD_STORAGE_CLASS": "1",
    "HAVE_ACCEPT_SOCKLEN_T": "1",
    "HAVE_ALIGNED_ALLOC": "1",
    "HAVE_ALIGNED_NEW": "1",
    "HAVE_ALLOW_POLL": "1",
    "HAVE_ALLOW_SELECT": "1",
    "HAVE_BYTESWAP_H": "1",
    "HAVE_ALLOW_CLICK_PACKET_POOL": "1",
    "HAVE_CLOCK_GETTIME": "1",
    "HAVE_DECL_CLOCK_GETTIME": "1",
    "HAVE_DECL_MADVISE": "1",
    "HAVE_DLFCN_H": "1",
    "HAVE_EXECINFO_H": "1",
    "HAVE_FLOW": "1",
    "HAVE_FFS": "1", "HAVE_FFSL": "1", "HAVE_FFSLL": "1",
    "HAVE_GRP_H": "1",
    "HAVE_IFADDRS_H": "1",
    "HAVE_INT64_IS_LONG_USERLEVEL": "1",
    "HAVE_INTTYPES_H": "1",
    "HAVE_LARGE_FILE_SUPPORT": "1",
    "HAVE_LINUX_ETHTOOL_H": "1", "HAVE_LINUX_SOCKIOS_H": "1", "HAVE_LINUX_IF_TUN_H": "1",
    "HAVE_LINUX_IF_PACKET_H": "1", "HAVE_LINUX_NETLINK_H": "1",
    "HAVE_MADVISE": "1",
    "HAVE_MMAP": "1",
    "HAVE_NETDB_H": "1",
    "HAVE_NETPACKET_PACKET_H": "1",
    "HAVE_NEW_HDR": "1",
    "HAVE_POLL_H": "1",
    "HAVE_PSELECT": "1",
    "HAVE_DECL_PTHREAD_SETAFFINITY_NP": "1",
    "HAVE_PWD_H": "1",
    "HAVE_RANDOM": "1",
    "HAVE_SIGACTION": "1",
    "HAVE_SNPRINTF": "1",
    "HAVE_STRERROR": "1",
    "HAVE_STRINGS_H": "1",
    "HAVE_STRNLEN": "1",
    "HAVE_STRTOF": "1", "HAVE_STRTOLD": "1", "HAVE_STRTOUL": "1",
    "HAVE_SYS_MMAN_H": "1",
    "HAVE_TCGETPGRP": "1",
    "HAVE_TERMIO_H": "1",
    "HAVE_U_INT_TYPES": "1",
    "HAVE_UNISTD_H": "1",
    "HAVE_USER_MULTITHREAD": "1",
    "HAVE_ATOMIC_BUILTINS": "1",
    "HAVE_VSNPRINTF": "1",
    "SIZEOF_OFF_T": "8",
}

_UNDEF = re.compile(r"^(\s*)#(\s*)undef\s+(\w+)\s*$")


def substitute(text: str, values: dict) -> str:
    """config.status's rule: `#undef NAME` -> `#define NAME VALUE` when NAME
    has a value, else `/* #undef NAME */`. Other lines are kept."""
    out = []
    for line in text.splitlines():
        m = _UNDEF.match(line)
        if m and m.group(3) != "inline":
            name = m.group(3)
            if name in values:
                line = f"{m.group(1)}#{m.group(2)}define {name} {values[name]}"
            else:
                line = f"{m.group(1)}/* #{m.group(2)}undef {name} */"
        out.append(line)
    return "\n".join(out) + "\n"


def generate(reference: str, out_dir: str) -> list[str]:
    click = os.path.join(out_dir, "click")
    os.makedirs(click, exist_ok=True)
    written = []
    for src, dst, values in (("config.h.in", "config.h", CONFIG_H),
                             ("config-userlevel.h.in", "config-userlevel.h", CONFIG_USERLEVEL_H)):
        with open(os.path.join(reference, src)) as f:
            text = substitute(f.read(), values)
        path = os.path.join(click, dst)
        with open(path, "w") as f:
            f.write(text)
        written.append(path)
    return written


if __name__ == "__main__":
    if len(sys.argv) != 3:
        raise SystemExit(__doc__)
    for p in generate(sys.argv[1], sys.argv[2]):
        print(p)
