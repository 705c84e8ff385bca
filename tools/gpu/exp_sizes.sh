#!/bin/bash
# Exponentiation kernel time against the item count per launch (wave packing), expchain probe V3 W2.
cd "$GRAFT_REPO_ROOT" || exit 1
for n in 65536 100000 131072 163840 200000 262144 300000 400000; do
  timeout -k 5 60 ./tools/microbench/expchain 11 $n 1 | tail -1 || exit 1
done
