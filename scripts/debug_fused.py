"""Debug helper (GPU box): one fused-counting pipeline call at bench size,
serialized, counters checked against torch.bincount of the outputs."""
import ctypes as C
import os
import sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vproxy_amd as V
from vproxy_amd import workloads as W
import bench as B

n = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000_000
dev = torch.device("cuda", 0)
clf = V.Classifier(0)
tcp, udp = W.gen_sg_rules(10000, W.SEED + 2, p_range=0.3)
a, na, ka = W.as_ctypes(tcp, V._lib.VcAclRule)
b, nb, kb = W.as_ctypes(udp, V._lib.VcAclRule)
V.check(V.lib().vc_compile_acl(clf.h, a, na, b, nb, 0))
net, plen = W.gen_v4_prefixes(1_000_000, W.SEED + 3)
rt = V.RouteTable()
allnets = W.v4_nets(net, plen)
arr, n_all, keep = W.as_ctypes(allnets, V._lib.VcNet)
rt.add_rules("bgp", arr, n=n_all)
clf.compile_route_table(rt)
n4 = rt.rules_raw(4)[1]
groups, ghosts = W.gen_groups(100_000, W.SEED + 5)
clf.compile_upstream(groups)
pool = torch.randint(-1, 100_000, (1 << 20,), dtype=torch.int32, device=dev)
proto, src, dst, dport, hid = B.gen_packets(n, tcp, udp, net, plen, 1 << 20, 5, dev)
torch.cuda.synchronize()
print("tables ready", flush=True)
clf.counters_enable(True)
clf.counters_reset()
acl, route, grp, _ = clf.pipeline_v4(proto, src, dst, dport, hid, pool)
torch.cuda.synchronize()
print("pipeline ok", flush=True)
cr = torch.from_numpy(clf.counters_read(V.COUNTERS_ROUTE).astype(np.int64))
exp = torch.bincount(torch.where(route >= 0, route, n4).long(), minlength=n4 + 2).cpu()
print("route counters equal:", bool(torch.equal(cr, exp)), flush=True)
cg = torch.from_numpy(clf.counters_read(V.COUNTERS_GROUP).astype(np.int64))
exp = torch.bincount(torch.where(grp >= 0, grp, 100_000).long(), minlength=100_001).cpu()
print("group counters equal:", bool(torch.equal(cg, exp)), flush=True)
