for t in 401 402 403 404; do
  JMH_BLOCK_PROF=$t timeout -k 10 200 python bench.py --steps 60 --no-cpu-baseline --no-host-path > /dev/null 2> gpurun_out/gap_$t.txt || exit 1
  grep "jmh_blocks tick" gpurun_out/gap_$t.txt | head -1 | cut -c1-400
done
