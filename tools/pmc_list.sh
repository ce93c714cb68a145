#!/bin/bash
# GPU box: the PMC counters rocprofv3 offers on this device whose names match a pattern.
# usage: tools/pmc_list.sh <regex>
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > /tmp/avail.txt 2>&1
grep -E -i "$1" /tmp/avail.txt | head -80
