import sys, time
sys.path.insert(0, '.')
from oracle import oracle as O
from prysm_amd import trieutil as T
deps = [bytes(O.splitmix_bytes(280, 5, 35 * i)) for i in range(4200)]
ref = T.DepositTrie(32, capacity=8192)
t = T.DepositTrie(32, capacity=8192)
for d in deps[:4096]:
    ref.update_deposit_trie(d); t.update_deposit_trie(d)
t.root()
logs = []
for d in deps[4096:4196]:
    logs.append((d, ref.root())); ref.update_deposit_trie(d)
t0 = time.perf_counter()
for d, r in logs:
    assert t.save_logs([d], [r]) == [True]
print("us per single-log save_logs", (time.perf_counter() - t0) / len(logs) * 1e6)
