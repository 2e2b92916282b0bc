#!/bin/sh
# Regenerates tests/golden/ from the reference's own code (see ref_harness.cc).
# Container-only: needs /root/reference.  TEST INFRASTRUCTURE ONLY.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
REF=${REF:-/root/reference}
GOLD="$HERE/../../tests/golden"
make -s -C "$HERE" REF="$REF"
mkdir -p "$GOLD"
"$HERE/../_ref/ref_harness" "$GOLD"
# coherent mode: the reference's MSI controllers in the canonical schedule
# (coh_harness.cc), plus configs[0]'s captured FFT trace (-m10 fixture)
python3 "$HERE/export_trace.py" "$GOLD/fft_real_p16_m10.npz" "$HERE/../_ref/fft10"
"$HERE/../_ref/coh_harness" "$GOLD" "$HERE/../_ref/fft10"
# the same schedule over the reference's MOSI controllers (coh_harness_mosi)
"$HERE/../_ref/coh_harness_mosi" "$GOLD" "$HERE/../_ref/fft10"
# the same schedule over the reference's shared-L2 MSI controllers (coh_harness_shl2)
"$HERE/../_ref/coh_harness_shl2" "$GOLD" "$HERE/../_ref/fft10"
# and over the shared-L2 MESI controllers (coh_harness_shl2_mesi)
"$HERE/../_ref/coh_harness_shl2_mesi" "$GOLD" "$HERE/../_ref/fft10"
