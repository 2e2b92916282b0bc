#!/bin/sh
# Regenerates tests/golden/ from the reference's own code (see ref_harness.cc).
# Container-only: needs /root/reference.  TEST INFRASTRUCTURE ONLY.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
REF=${REF:-/root/reference}
make -s -C "$HERE" REF="$REF"
mkdir -p "$HERE/../../tests/golden"
"$HERE/../_ref/ref_harness" "$HERE/../../tests/golden"
# coherent mode: the reference's MSI controllers in the canonical schedule (coh_harness.cc)
"$HERE/../_ref/coh_harness" "$HERE/../../tests/golden"
