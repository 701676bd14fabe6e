export GPU_MAX_HW_QUEUES=16
for r in 1 2; do for lib in ab/l1.so ab/l2.so; do
  f=$(FD_AMD_LIB=$PWD/$lib timeout -k 10 120 python3 tools/lat_floor.py 2>/dev/null | grep -E "^(16384|4096) " | python3 -c "import sys,json; print(' '.join('%s:%.4f' % (l.split()[0], json.loads(l.split(' ',1)[1])['k_dsm']) for l in sys.stdin))") || exit 1
  echo "$lib k_dsm ms $f"
done; done
