#!/bin/sh
# Regenerate the golden vectors from the real reference (eromero-vlc/superbblas, header-only,
# built from /root/reference by oracle/Makefile with the OpenBLAS bundled in this image).
# SB_DEBUG=2 turns on the reference's own mock-index self-check of every copy (dist.h:1919-2116).
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
make -C "$HERE/../../oracle" ref
rm -f "$HERE"/case*.bin "$HERE"/manifest.jsonl
OMP_NUM_THREADS=4 OPENBLAS_NUM_THREADS=1 SB_DEBUG=2 "$HERE/../../oracle/_ref/ref_golden" "$HERE"
