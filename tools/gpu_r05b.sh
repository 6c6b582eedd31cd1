#!/bin/bash
# issue-cost lab (tools/lab/issue_lab.hip, prebuilt in tools/lab/bin)
set -o pipefail
OUT=gpurun_out/r05b
mkdir -p $OUT
timeout -k 10 120 tools/lab/bin/issue_lab > $OUT/issue_lab.txt 2>&1; rc=$?
cat $OUT/issue_lab.txt; exit $rc
