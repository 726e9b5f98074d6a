#!/bin/bash
# Build the QR-tree oracle from the reference's tree sources (read-only; compiled here, nothing prebuilt).
set -e
D=$(cd "$(dirname "$0")" && pwd)
REF=${REF:-/root/reference/src}
gcc -O1 -std=gnu99 -w -I"$D/stub" -I"$REF/include" -o "$D/oracle" "$D/oracle.c" "$REF/dplasma_hqr.c" \
    "$REF/dplasma_systolic_qr.c" -lm
echo "$D/oracle"
