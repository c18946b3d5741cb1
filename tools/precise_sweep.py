"""precise-mode throughput at several shard counts / staggers (bench.precise_mode), one process:
python tools/precise_sweep.py "2:1,2:2,3:2,1:0" """
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts-zs_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from stzs.params import init_params  # noqa: E402
from stzs.spec import SPEC_V0 as S  # noqa: E402

P = init_params(S, 0)
for spec in (sys.argv[1] if len(sys.argv) > 1 else "2:1,2:2,3:2").split(","):
    ns, sg = (int(v) for v in spec.split(":"))
    r = bench.precise_mode(S, P, "cuda:0", nstream=ns, stagger=sg)
    print(f"precise {ns} shards stagger {sg}: {r['audio_s_per_s']} audio-s/s ({r['ms_per_step']} ms/step; one stream "
          f"{r['single_stream_audio_s_per_s']})", flush=True)
    torch.cuda.empty_cache()
