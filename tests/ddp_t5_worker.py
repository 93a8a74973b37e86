"""One rank of the 2-process T5-overlap GPU test (tests/test_ddp_gpu.py); both ranks share the one
GPU and talk over gloo, in deterministic mode (MMT_DETERMINISTIC=1). Not collected by pytest.

The bench's N > 1 step (distributed.DDPStep: staged backward graphs, each stage's gradient region
all-reduced asynchronously) with the frozen T5 encoder of the next step overlapped (txt_next) and
without it, from the same parameters, over steps whose text changes every step: the parameters
after the steps must be equal bit for bit (the overlap changes only where the encoder runs).
Writes a JSON report to argv[1].
"""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_path = sys.argv[1]
    from multi_modal_transformers_tokenmerge_amd.distributed import DDPStep, GradAllReducer, init_from_env
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.models.octo.octo import Octo, create_octo_train_state
    from multi_modal_transformers_tokenmerge_amd.tokenizers.text.t5_base import T5Config
    from oracle.parity import _inputs
    di = init_from_env(backend="gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, N, steps = 2, di.world_size, 3
    cfg = get_config("octo-small-tome16", num_blocks=2, t5=T5Config(num_layers=2))
    sl = slice(di.rank * B, (di.rank + 1) * B)
    model0 = Octo(cfg, dev, seed=0)
    batches = []
    for i in range(steps + 1):
        images, text, actions = _inputs(model0, N * B, seed=50 + i)
        batches.append(tuple(torch.from_numpy(x)[sl].contiguous().to(dev) for x in (images, text, actions)))
    model0.store.set_deterministic(False)   # one ParamStore holds the mode at a time

    def run(overlap):
        model = Octo(cfg, dev, seed=0)
        red = GradAllReducer(N, bucket_bytes=1 << 20)
        state = create_octo_train_state(model, seed=11, allreduce=red, sample_offset=di.rank * B)
        img, txt, act = (x.clone() for x in batches[0])
        txt_next = batches[1][1].clone()
        step = DDPStep(model, state, txt, img, act, red, stages="auto:0.001", use_graph=True,
                       txt_next=txt_next if overlap else None).build(warm=1)
        for i in range(steps):
            img.copy_(batches[i][0]); txt.copy_(batches[i][1]); act.copy_(batches[i][2])
            txt_next.copy_(batches[i + 1][1])
            step()
        torch.cuda.synchronize()
        res = model.store.flat.clone(), float(step.loss_buf), step.S, step.t5_pf
        model.store.set_deterministic(False)
        return res

    p_on, loss_on, S, pf_on = run(True)
    p_off, loss_off, _, pf_off = run(False)
    rep = dict(rank=di.rank, stages=S, overlap_on=pf_on, overlap_off=not pf_off,
               params_bitwise=bool(torch.equal(p_on, p_off)), loss_on=loss_on, loss_off=loss_off)
    dist.barrier()
    dist.destroy_process_group()
    with open(out_path, "w") as f:
        json.dump(rep, f)
    print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
