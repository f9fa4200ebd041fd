"""FETCH_SIZE calibration for the filter's access pattern:
the config-2 filter plan with a predicate no row passes reads exactly the two
predicate columns (id i32 + price f64 = 12 B per row, every line once) and
writes nothing, so FETCH_SIZE per launch / (12 n) is the correction factor
for this access on gfx950.  Run under rocprofv3 --pmc FETCH_SIZE WRITE_SIZE."""
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0] + "/flink-siddhi_amd")
import flink_siddhi as fs  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 26
plan = ("define stream inputStream (id int, name string, price double, timestamp long);"
        "from inputStream[price > 2.0 and id % 7 == 0] select * insert into O;")
rt = fs.SiddhiAppRuntime(plan)
rt.add_callback("O")
g = torch.Generator(device="cuda").manual_seed(1)
ids = torch.randint(0, 1000, (n,), dtype=torch.int32, device="cuda", generator=g)
price = torch.rand(n, dtype=torch.float64, device="cuda", generator=g)
ts = torch.arange(n, dtype=torch.int64, device="cuda")
names = torch.zeros(n, dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
for _ in range(3):
    rt.send("inputStream", ts, [ids, names, price, ts])
    rt.flush()
assert len(rt.collect("O")) == 0
print("calibration: %d rows, %d predicate bytes per launch" % (n, 12 * n))
