#!/bin/bash
# round 5 job zh: the BERT-feature prefetch stream at high priority (IRC_HIGH_PRIORITY_STREAMS=
# bert_prefetch) against the default, whole bench (every leg in one process), interleaved twice:
# does the pipelined retrieval still slow down now that it runs without HIP graphs?
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in def hp; do
    if [ $v = hp ]; then export IRC_HIGH_PRIORITY_STREAMS=bert_prefetch; else unset IRC_HIGH_PRIORITY_STREAMS; fi
    timeout -k 10 500 python bench.py --no-cpu-baseline > gpurun_out/r5_zh_${v}_$i.log 2>&1 || exit $?
    cp gpurun_out/bench_detail.json gpurun_out/r5_zh_${v}_$i.json
    python3 -c "
import json; d=json.load(open('gpurun_out/r5_zh_${v}_$i.json'))
print('$v $i', 'train', round(d['train']['pairs_per_s']), 'c2', round(d['retrieval']['value']), 'c3', round(d['retrieval_c3']['value']), 'c4', round(d['retrieval_c4']['value']), 'fp8', round(d['retrieval_fp8']['value']), 'bert', round(d['train_bert']['pairs_per_s']))"
  done
done
