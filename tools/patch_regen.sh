#!/bin/bash
# Regenerate an integration patch from an edited copy of the reference files.
#   tools/patch_regen.sh open  <patch> <dir> <relpath>...   copy the files from /root/reference into <dir>/a and
#                                                           <dir>/b, apply <patch> to <dir>/b (edit <dir>/b next)
#   tools/patch_regen.sh write <patch> <dir> <relpath>...   rewrite <patch> as the diff a -> b, in argument order
set -e
mode=$1; patch=$(realpath "$2"); dir=$3; shift 3
if [ "$mode" = open ]; then
  rm -rf "$dir"; mkdir -p "$dir/a" "$dir/b"
  for f in "$@"; do
    mkdir -p "$dir/a/$(dirname "$f")" "$dir/b/$(dirname "$f")"
    cp "/root/reference/$f" "$dir/a/$f"; cp "/root/reference/$f" "$dir/b/$f"; chmod u+w "$dir/b/$f"
  done
  (cd "$dir/b" && patch -s -p1 < "$patch")
else
  : > "$patch.new"
  for f in "$@"; do
    (cd "$dir" && diff -u --label "a/$f" --label "b/$f" "a/$f" "b/$f" >> "$patch.new") || [ $? -eq 1 ]
  done
  mv "$patch.new" "$patch"
fi
