"""One line per PS bench log: ms/update, PS host us per message by phase, and per worker
(push us, reply wait us, pull us, compute us)."""
import json
import sys

tag, path = sys.argv[1], sys.argv[2]
d = json.loads([l for l in open(path) if l.startswith('{"metric')][-1])
print(tag, d["ms_per_update"], d["ps_us_per_msg"],
      [(c["push_us"], c["reply_wait_us"], c["pull_us"], c.get("compute_us")) for c in d["ps_comm"]])
