# quick bucketed-build check on the GPU (round-4 bring-up): a few shapes vs the oracle
import os, sys
os.environ["ADL_BLOOM_DEBUG"] = "1"
sys.path.insert(0, "adlsm-tree_amd"); sys.path.insert(0, "oracle")
import numpy as np, torch, adlbloom, oracle
def chk(name, keys_dev, bpk=10):
    bm = adlbloom.build(keys_dev, bits_per_key=bpk).cpu().numpy()
    ok = np.array_equal(bm, oracle.keys2block(keys_dev.cpu().numpy(), bits_per_key=bpk))
    print(name, "equal" if ok else "DIFF", flush=True)
    return ok
ok = chk("n=20000", adlbloom.synth_keys16(20000, seed=0x5EED))
ok = ok and chk("n=1000000", adlbloom.synth_keys16(1000000, seed=0x5EED))
ok = ok and chk("n=5 bpk=1", adlbloom.synth_keys16(5, seed=3), bpk=1)
base = adlbloom.synth_keys16(7, seed=1).cpu().numpy()
ok = ok and chk("dup 7x20000", torch.from_numpy(np.repeat(base, 20000, axis=0)).cuda())
ok = ok and chk("n=3000000 bpk=20", adlbloom.synth_keys16(3000000, seed=9), bpk=20)
if ok:
    data, offs = adlbloom.synth_varlen(300_000, seed=0x5EED)
    bm = adlbloom.build(data, offs).cpu().numpy()
    ok = np.array_equal(bm, oracle.keys2block(data.cpu().numpy(), offs.cpu().numpy().view(np.uint64)))
    print("varlen 300k", "equal" if ok else "DIFF", flush=True)
if ok:
    # segmented var-len, 13 filters (descriptor table), empty and 1-key filters
    sizes = [0, 1, 511, 512, 513, 40000, 7, 0, 1, 90000, 3, 1025, 20000]
    data, offs = adlbloom.synth_varlen(sum(sizes), seed=77)
    kb = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    out, boff, nbytes = adlbloom.build_segmented(data, kb, offsets=offs)
    out = out.cpu().numpy(); hd = data.cpu().numpy(); ho = offs.cpu().numpy().view(np.uint64)
    for f in range(len(sizes)):
        o = ho[int(kb[f]):int(kb[f + 1]) + 1]
        want = oracle.keys2block(hd, o - o[0] if False else o, bits_per_key=10) if False else None
        ks = [hd[int(ho[i]):int(ho[i + 1])].tobytes() for i in range(int(kb[f]), int(kb[f + 1]))]
        want = oracle.keys2block(ks)
        got = out[int(boff[f]):int(boff[f]) + int(nbytes[f])]
        if not np.array_equal(got, want):
            ok = False
            print("seg varlen filter", f, "DIFF", flush=True)
    print("seg varlen 13 filters", "equal" if ok else "DIFF", flush=True)
if ok:
    keys = adlbloom.synth_keys16(10_000_000, seed=0x5EED)
    b = adlbloom.Builder(10_000_000, 10)
    for i in range(3):
        b.build(keys)
    torch.cuda.synchronize()
    import time
    t0 = time.time()
    for i in range(20):
        b.build(keys)
    torch.cuda.synchronize()
    dt = (time.time() - t0) / 20
    print("10M build ms", dt * 1e3, "Gkeys/s", 10e6 / dt / 1e9, flush=True)
    print("10M equal", np.array_equal(b.build(keys).cpu().numpy(), oracle.keys2block(keys.cpu().numpy())))
