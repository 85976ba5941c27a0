"""One rank of the world-size-2 rehearsal (tests/test_gpu_dist.py): the batch
is sharded by rank exactly as bench.py shards it, every rank runs the HIP
library on its own shard, and rank 0 checks that the gathered shard outputs
equal the single-process result over the whole batch.  gloo carries only
the check's gather (the product path has no collective)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ntt-gpu-qtesla_amd"))
sys.path.insert(0, ROOT)


def main(out_path):
    import torch
    import torch.distributed as dist
    import ntt_amd
    from bench import shard

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    res = {}
    for ps, per_rank in (("p-III", 3001), ("p-I", 2999)):   # odd: the n=1024 half-wave tail on every rank
        n = ntt_amd.param_info(ps)["n"]
        first, count = shard(per_rank, rank)
        x = torch.empty(count * n, dtype=torch.int32, device=dev)
        y = torch.empty_like(x)
        ntt_amd.fill_uniform(x, ps, 0xD157, first)
        ntt_amd.fill_uniform(y, ps, 0xD158, first)
        z = torch.empty_like(x)
        ntt_amd.poly_mul(z, x, y, ps)
        ntt_amd.poly_ntt(x, ps)
        torch.cuda.synchronize(dev)
        outs = {}
        for name, t in (("ntt", x), ("mul", z)):
            parts = [torch.empty(count * n, dtype=torch.int32) for _ in range(world)]
            dist.all_gather(parts, t.cpu())
            outs[name] = torch.cat(parts)
        if rank == 0:
            total = world * per_rank
            fx = torch.empty(total * n, dtype=torch.int32, device=dev)
            fy = torch.empty_like(fx)
            ntt_amd.fill_uniform(fx, ps, 0xD157, 0)
            ntt_amd.fill_uniform(fy, ps, 0xD158, 0)
            fz = torch.empty_like(fx)
            ntt_amd.poly_mul(fz, fx, fy, ps)
            ntt_amd.poly_ntt(fx, ps)
            res[ps] = {"ntt": bool(torch.equal(outs["ntt"], fx.cpu())), "mul": bool(torch.equal(outs["mul"], fz.cpu())),
                       "world": world, "per_rank": per_rank}
    dist.barrier()
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
