#!/bin/bash
# Build the FastClick package element against an installed FastClick when
# one is given (CLICKPREFIX, default /usr/local). Without one there is
# nothing to compile against: say so and succeed.
cd "$(dirname "$0")"
P=${CLICKPREFIX:-/usr/local}
if [ ! -r "$P/share/click/config.mk" ]; then
  echo "fastclick_pkg: no FastClick install under $P (share/click/config.mk); element not built"
  exit 0
fi
make CLICKPREFIX="$P"
