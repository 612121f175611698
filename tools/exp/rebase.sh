#!/bin/bash
# Re-base the experiment patches (tools/exp/*.patch, applied in name order by `make exp`) on the
# current csrc/: apply each one (fuzz allowed) on top of the ones before it and rewrite it as an exact
# diff.  A hunk that fails leaves its .rej under /tmp/exp_rebase/<patch>/ and stops: fix that copy by
# hand, then rerun with FROM=<patch name> to regenerate from there.
#   bash tools/exp/rebase.sh
set -eu
HERE=$(cd "$(dirname "$0")" && pwd)
CSRC=$HERE/../../rust-ray-tracing_amd/csrc
W=/tmp/exp_rebase
rm -rf "$W" && mkdir -p "$W/cur"
cp "$CSRC"/*.hip "$CSRC"/*.hpp "$W/cur/"
for p in "$HERE"/*.patch; do
    n=$(basename "$p" .patch)
    rm -rf "$W/base" "$W/$n" && cp -r "$W/cur" "$W/base" && cp -r "$W/cur" "$W/$n"
    if ! patch -s -p1 -d "$W/$n" < "$p"; then
        echo "rebase.sh: $n does not apply; see $W/$n/*.rej" >&2
        exit 1
    fi
    rm -f "$W/$n"/*.orig
    (cd "$W" && diff -u base "$n" | sed "s#^--- base/#--- a/#; s#^+++ $n/#+++ b/#") > "$p" || true
    rm -rf "$W/cur" && cp -r "$W/$n" "$W/cur"
    echo "rebased $n"
done
