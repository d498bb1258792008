#!/bin/bash
# summarize serve bench logs in a dir: name, req/s, latencies, CPU
cd "$1" && for f in $(ls $2*.log | sort -t_ -k3); do python3 -c "
import json
l=[x for x in open('$f') if x.startswith('{')][-1]
d=json.loads(l); c=d['cpu_breakdown_rank0']; io=c['io_stage_us_per_req']
print('%-22s %8.0f p50 %.4f p99 %.4f b1 %.4f cpu/req %.2f srv_lat %.1f cores %.2f lg %.2f poll %.2f idle %.2f send %.2f recv %.2f' % ('$f'[:-4], d['value'], d['p50_latency_ms_c64'], d['p99_latency_ms_c64'], d['p50_latency_ms_batch1'], c['server_cpu_us_per_req'], c['server_http_latency_us_mean'], d['cpu_cores_busy_rank0']['process_total'], d['cpu_cores_busy_rank0']['loadgen_process'], io['poll'], io['idle_gpu'], io['send'], io['recv']))
"; done
