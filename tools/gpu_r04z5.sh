# round-4 GPU pass: 256-row epilogue aux ring of 4 row groups (CLIPK_XBUD256=32, build_ab/xb32)
# vs 2 (default 16): headline site table, interleaved
set -o pipefail
mkdir -p gpurun_out
for v in base xb32 base xb32; do
  echo "== $v" >> gpurun_out/r04z5_sites.txt
  if [ $v = xb32 ]; then export CLIPK_LIB=build_ab/xb32/libclipk.so; else unset CLIPK_LIB; fi
  timeout -k 10 300 python -u tools/site_table.py 2>&1 | grep -E "sum of|dgelu|fc_fwd|proj_fwd|out_fwd" >> gpurun_out/r04z5_sites.txt || exit 1
done
echo exit 0
