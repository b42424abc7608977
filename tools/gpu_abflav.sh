#!/bin/bash
# Same-box A/B of library flavours (libshdtopology_<name>.so, "prod" = libshdtopology.so),
# interleaved: LIBS="prod oob" WL="cfg5 cfg4" REPS_LIB=2 PASSES=2 [CONF="ENV=V"] [TAG=x].
# Logs under gpurun_out/abflav[_TAG].log.
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/abflav${TAG:+_$TAG}.log
: > "$L"
for r in $(seq 1 "${REPS_LIB:-2}"); do
  for wl in ${WL:-cfg5 cfg4}; do
    for lib in ${LIBS:-prod oob}; do
      v=$lib; [ "$lib" = prod ] && v=""
      echo "### rep $r $wl lib=$lib" >> "$L"
      SHDR_LIB_VARIANT=$v REPS=1 PASSES=${PASSES:-2} timeout -k 10 300 python -u tools/ab.py "$wl" "${CONF:-}" >> "$L" 2>&1 || { echo "ab $wl $lib failed"; tail -20 "$L"; exit 9; }
    done
  done
done
grep -E "^###|warm mean" "$L"
