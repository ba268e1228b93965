"""Probe: create a CU-masked stream (hr_stream_create_cu_mask), use it from torch (ExternalStream), destroy it
(hr_stream_destroy), exit.  Variant `plain`: caching-allocator blocks made on the stream; `embed`: the query embedder's
graphed forward on it (the bench's CU split); `search`: a ShardedSearch batch with the scan on it.  Prints the stage
reached; the parent reads the exit status (an abort at exit after destroying such a stream)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "youtu-rag_amd")]


def main(variant: str, destroy_mode: str, alive: bool = False) -> None:
    import torch

    from hiprag import _native

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    raw = _native.create_cu_stream(0, range(0, 128))
    es = torch.cuda.ExternalStream(raw, device=dev)
    keep = []
    if variant == "plain":
        with torch.cuda.stream(es):
            x = torch.randn(1 << 20, device=dev)
            keep.append((x * 2).sum())
    elif variant == "embed":
        from hiprag.rag.rocm_embedder import TorchRocmEmbedder

        emb = TorchRocmEmbedder(preset="tiny", dtype="bfloat16", device=dev, batch_size=16)
        for _ in range(3):
            with torch.cuda.stream(es):
                keep.append(emb.embed_queries_device([f"query {i} about things" for i in range(16)]).sum())
    elif variant == "split":  # the bench's CU split: embedder on one masked stream, scan + tail on two others
        from hiprag.dist import ShardedSearch
        from hiprag.rag.rocm_embedder import TorchRocmEmbedder

        n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
        e_cus = list(range(0, n_cu, 4))
        s_cus = [c for c in range(n_cu) if c % 4]
        emb = TorchRocmEmbedder(preset="tiny", dtype="bfloat16", device=dev, batch_size=16)
        idx = _native.NativeIndex(256, "bf16", "cosine")
        idx.add_synthetic(0, 0, 200_000)
        ss = ShardedSearch(idx, 0, max_batch=16, device=dev)
        _native.destroy_stream(raw)
        raw_l = [_native.create_cu_stream(0, e_cus), _native.create_cu_stream(0, s_cus), _native.create_cu_stream(0, s_cus)]
        es, scan, tail = (torch.cuda.ExternalStream(r, device=dev) for r in raw_l)
        tail0 = ss.tail
        idx.set_cu_mask(s_cus)
        ss.tail = tail
        s_out = torch.empty((4, 16, 10), device=dev)
        r_out = torch.empty((4, 16, 10), dtype=torch.int64, device=dev)
        for i in range(4):
            with torch.cuda.stream(es):
                q = emb.embed_queries_device([f"query {i} {j}" for j in range(16)])
                ev = torch.cuda.Event()
                ev.record(es)
            keep.append((q, ev))
            scan.wait_event(ev)
            with torch.cuda.stream(scan):
                ss.submit(q, 10, s_out=s_out[i], r_out=r_out[i], q_ready=ev)
        ss.finalize_all()
        torch.cuda.synchronize()
        ss.tail = tail0
        idx.set_cu_mask(None)
        keep.append(s_out.sum())
        torch.cuda.synchronize()
        print("used", flush=True)
        if destroy_mode == "lib":
            for r in raw_l:
                _native.destroy_stream(r)
        print("destroyed", flush=True)
        if not alive:
            del keep, q, ev
        return
    elif variant == "search":
        from hiprag.dist import ShardedSearch

        idx = _native.NativeIndex(256, "bf16", "cosine")
        idx.add_synthetic(0, 0, 200_000)
        ss = ShardedSearch(idx, 0, max_batch=16, device=dev)
        q = torch.randn((16, 256), device=dev)
        with torch.cuda.stream(es):
            s, r = ss.search(q, 10)
            keep.append(s.sum())
        ss.close()
    es.synchronize()
    print("used", [float(v) for v in keep], flush=True)
    if not alive:
        del keep  # (alive: the tensors made on the stream outlive it, freed at interpreter exit)
    if destroy_mode == "lib":
        _native.destroy_stream(raw)
    print("destroyed", flush=True)
    globals()["_keep_alive"] = keep if alive else None


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "lib", len(sys.argv) > 3 and sys.argv[3] == "alive")
    print("exiting", flush=True)
