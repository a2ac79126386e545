#!/bin/bash
# fqz5file on a 1 GB file (the dropin item's CRC failure), the -5 decode
# regression A/B (register decoder / XCD grouping), the fqz decoder
# set-address multiply A/B.
set -uo pipefail
OUT=gpurun_out/ab5
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/file_path_check.py 1.0 3 > $OUT/file.log 2>&1
echo "file rc=$?"; tail -3 $OUT/file.log
B5="--no-cpu --no-crc --no-dropin --level 5 --kind novaseq --gb 4 --steps 4 --warmup 1"
for v in def noreg noxcd; do
  case $v in noreg) export FQZ5_NO_REGDEC=1;; noxcd) unset FQZ5_NO_REGDEC; export FQZ5_NO_XCD_GROUP=1;; esac
  timeout -k 10 300 python3 bench.py $B5 > $OUT/b5$v.json 2> $OUT/b5$v.log || { echo "b5 $v failed"; tail -5 $OUT/b5$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b5$v.json'));print('$v',d['value'],d['enc_ms_per_step'],d['dec_ms_per_step'],d['roofline']['dec_avg_ms'])"
done
unset FQZ5_NO_XCD_GROUP
timeout -k 10 200 python3 -u tools/fqz_timing.py 60000 15000 > $OUT/fqz_new.log 2>&1; tail -6 $OUT/fqz_new.log
FQZ5_LIB_VARIANT=tools/vtmp/libfqz5_old.so timeout -k 10 200 python3 -u tools/fqz_timing.py 60000 15000 > $OUT/fqz_old.log 2>&1; tail -6 $OUT/fqz_old.log
