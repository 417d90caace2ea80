cd ${GRAFT_REPO_ROOT}
OUT=gpurun_out/$S_OUT; mkdir -p $OUT
for rep in 1 2; do for v in $VALS; do
  if [ "$v" = default ]; then lib=""; else lib=$PWD/real-time-gpu-ray-tracer_amd/lib/librtamd_$v.so; fi
  RTAMD_LIB=$lib timeout -k 10 200 python3 scripts/rebuild_alone.py --updates 30 > $OUT/rb_${v}_$rep.log 2>&1 || { echo "$v failed"; tail -5 $OUT/rb_${v}_$rep.log; exit 1; }
  echo "$v $(tail -1 $OUT/rb_${v}_$rep.log)"
done; done
