import sys
sys.path[:0] = ['scalecube-cluster_amd', 'oracle', 'tests', 'tests/golden']
import scenarios, swimgpu, oracle
from swimgpu import abi
sc = [s for s in scenarios.catalog() if s.name == "join_burst_seg"][0]
for name, lib in (("oracle", oracle.lib()), ("gpu", swimgpu.load_library())):
    e = scenarios.make_engine(lib, sc)
    mx = [0, 0]
    def chk(t):
        g = max(e.read_member(m)["gossip_len"] for m in range(sc.capacity))
        if g > mx[0]: mx[0], mx[1] = g, t
    sc.check_every = 5
    try:
        scenarios.run(e, sc, chk)
        print(name, "ok max gossip_len", mx, flush=True)
    except abi.SwimError as ex:
        print(name, "error", ex, hex(e.stats()["capacity_errors"]), "max gossip_len", mx, "at tick", e.now()[0], flush=True)
