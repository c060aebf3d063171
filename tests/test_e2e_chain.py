"""BASELINE config 3 end to end on the GPU: frames -> detectron2 Faster R-CNN X101-32x8d-FPN person detection -> the
single-person gate (mesh_generator.py:101-117) -> ViTDetDataset crops -> TokenHMR (ViT-H width); YOLOX-L persons ->
DWPose (RTMPose-l, every frame) -> npz / keypoints.npy files (extract_mesh.py:35-43, process_video.py:59-94) -> the
scorer (featurise -> encoder -> AC/TC, eval.py:350-466), each stage checked against its oracle on the chain's own data:

  gate detector the Faster R-CNN's gate count and person box on two of the chain's frames vs oracle/frcnn.py's whole
                predictor (the stage-by-stage parity is tests/test_frcnn.py)
  gate          which videos are kept and which frames, the reference's 80 % rule on the detector's output
  crops         byte-identical to oracle/hmr.py vitdet_crop around the gate's person boxes
  TokenHMR      pose / global_orient / betas / token rows vs oracle/hmr.py at the extractor tests' tolerances
  DWPose        YOLOX-L anchor scores vs oracle/yolox.py, the two persons = greedy NMS on the GPU's anchors, SimCC
                logits vs oracle/dwpose.py; keypoints.npy rows = the oracle's composition of the decoded points
  scoring       the files the chain wrote, scored by vge.eval.run_eval and by oracle/evalflow.py's restatement of
                eval.py: AC / TC within 1e-4 (the north star), video set and keys equal

Parity of the networks vs the upstream TokenHMR / detectron2 / DWPose weights is UNPINNED (third-party code and
weights absent offline, random weights here).  TokenHMR runs 2 of ViT-H's 32 blocks (full
width, full decoder) so the CPU oracle finishes in seconds; the Faster R-CNN, RTMPose-l and YOLOX-L run at full size.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
C, T = 6, 12          # clips x frames: clips 0-4 carry 1-2 frames without exactly one person (kept), clip 5 carries 4
BAD = (1, 2, 1, 2, 1, 4)


@pytest.fixture(scope="module")
def chain(golden_dataset, tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vge import synth
    from vge.dwpose import RTMPOSE_L, YOLOX_L, DwposeExtractor, YoloxDetector
    from vge.extract import gate_mask, save_video_npz, single_person_frames
    from vge.frcnn import FRCNN_X101, FrcnnDetector
    from vge.hmr import HmrConfig, HmrExtractor, crop_persons
    root = tmp_path_factory.mktemp("e2e")
    hcfg = HmrConfig(depth=2)
    hsd = synth.make_hmr_state_dict(hcfg)
    fsd = synth.make_gate_frcnn_state_dict(FRCNN_X101)
    ysd = synth.make_gate_detector_state_dict(YOLOX_L)
    psd = synth.make_rtmpose_state_dict(RTMPOSE_L)
    gdet = FrcnnDetector(fsd, FRCNN_X101, device=DEV, chunk=32)
    det = YoloxDetector(ysd, YOLOX_L, device=DEV, chunk=64)
    hmr = HmrExtractor(hsd, hcfg, device=DEV, max_frames=C * T)
    pose = DwposeExtractor(psd, RTMPOSE_L, device=DEV, max_instances=2 * C * T)

    # the clips' frames from a pool of synthetic scenes, by what the gate detector finds in each (as the e2e bench does)
    pool = torch.from_numpy(synth.make_frame_pool(4242, 512)).to(DEV)
    one = gate_mask(gdet.detect(pool)["n_person"].cpu().numpy())
    good, bad = np.flatnonzero(one), np.flatnonzero(~one)
    assert good.size >= C * T and bad.size >= sum(BAD), (good.size, bad.size)
    rs = np.random.default_rng(5)
    idx = np.concatenate([rs.permutation(np.concatenate([rs.choice(bad, nb, replace=False),
                                                         rs.choice(good, T - nb, replace=False)])) for nb in BAD])
    frames = pool[torch.from_numpy(idx).to(DEV)].contiguous()
    del pool

    # the chain: gate detection -> gate -> crops -> TokenHMR; YOLOX persons -> DWPose on every frame (process_video.py
    # has no gate)
    g = {k: v.cpu().numpy() for k, v in gdet.detect(frames).items()}
    gboxes = g["person"][:, 0, :4]
    keep = gate_mask(g["n_person"])
    kept = {c: single_person_frames(np.where(keep[c * T:(c + 1) * T], 1, 0)) for c in range(C)}
    acc = [c for c in range(C) if kept[c] is not None]
    fidx = np.concatenate([c * T + kept[c] for c in acc])
    crops = crop_persons(frames, gboxes[fidx], fidx)
    cand = torch.empty((C * T, det.anchors, 5), device=DEV)
    boxes, npers, scores = det.detect(frames, cand=cand, with_scores=True)
    boxes, npers, scores = boxes.cpu().numpy(), npers.cpu().numpy(), scores.cpu().numpy()
    mesh = {k: v.cpu().numpy() for k, v in hmr.extract(crops).items()}
    K, WXY = RTMPOSE_L.keypoints, RTMPOSE_L.split * (RTMPOSE_L.in_w + RTMPOSE_L.in_h)
    n_inst = pose.instances(npers)
    simcc = torch.empty((n_inst, K, WXY), device=DEV)
    lv = torch.empty((n_inst, K, 3), device=DEV)
    rows = pose.keypoints(frames, boxes, npers, simcc=simcc, lv=lv).cpu().numpy()

    # the on-disk hand-off the reference's scripts make: one npz per accepted video (its kept frames), keypoints.npy
    # for every video, in the generated-set layout eval.py reads (flat meshes, flat keypoint dirs)
    gen, gkp = root / "generated_meshes", root / "generated_kps"
    from vge.data import ACTION_CLASSES
    classes = ACTION_CLASSES[:C]           # the golden real set's classes: every accepted video gets an AC score
    stems = [f"vgen_{classes[c]}_{c:02d}" for c in range(C)]
    j = 0
    for c in acc:
        n = kept[c].size
        info = {int(f): {"pose": mesh["pose"][j + a].reshape(23, 3, 3), "betas": mesh["betas"][j + a],
                         "global_orient": mesh["global_orient"][j + a].reshape(1, 3, 3), "vit": mesh["vit"][j + a]}
                for a, f in enumerate(kept[c])}
        save_video_npz(stems[c], info, out_root=gen, meta={"action": classes[c], "video": stems[c] + ".mp4"})
        j += n
    for c in range(C):
        d = gkp / stems[c]
        d.mkdir(parents=True)
        np.save(d / "keypoints.npy", rows[c * T:(c + 1) * T].astype(np.float32))
    gdet.close()
    return dict(frames=frames.cpu().numpy(), cand=cand.cpu().numpy(), boxes=boxes, npers=npers, scores=scores,
                gate=g, gboxes=gboxes, keep=keep, kept=kept, acc=acc, fidx=fidx, crops=crops.cpu().numpy(), mesh=mesh,
                rows=rows, simcc=simcc.cpu(), lv=lv.cpu(), hcfg=hcfg, hsd=hsd, fsd=fsd, ysd=ysd, psd=psd, gen=str(gen),
                gkp=str(gkp), stems=stems, paths=golden_dataset[0], ckpt=golden_dataset[1])


def test_gate_detector_and_gate(chain):
    """The Faster R-CNN's gate count and person box on two of the chain's frames (one kept, one not) vs the oracle's
    whole predictor (unless an oracle person score lies within 0.05 of 0.5), then the 80 % rule."""
    from oracle.frcnn import OracleFrcnn, gate_persons
    from vge.frcnn import FRCNN_X101
    g = chain["gate"]
    f_keep, f_drop = int(np.flatnonzero(chain["keep"])[0]), int(np.flatnonzero(~chain["keep"])[0])
    torch.set_num_threads(16)
    res = OracleFrcnn(chain["fsd"], FRCNN_X101, bf16=True).detect(chain["frames"][[f_keep, f_drop]])
    for r, f in zip(res, (f_keep, f_drop)):
        ps = r["scores"][r["classes"] == 0]
        print(f"frame {f}: persons > 0.5 gpu {int(g['n_person'][f])} oracle {gate_persons(r)}, "
              f"oracle person scores {ps[:3].tolist()}")
        if bool(((ps - 0.5).abs() < 0.05).any()):
            continue
        assert int(g["n_person"][f]) == gate_persons(r)
        if gate_persons(r) == 1:
            b = r["boxes"][r["classes"] == 0][0].numpy()
            np.testing.assert_allclose(chain["gboxes"][f], b, atol=2.0)
    # the 80 % rule (mesh_generator.py:113-117): clips 0-4 lose 1-2 frames and are kept, clip 5 is rejected
    assert chain["acc"] == [0, 1, 2, 3, 4]
    for c in chain["acc"]:
        assert chain["kept"][c].size == T - BAD[c]


def test_dwpose_detector(chain):
    """DWPose's own YOLOX-L persons (process_video.py's Wholebody): anchor scores vs the oracle, and the two persons
    the pose model reads = the greedy NMS on the GPU's anchors."""
    from oracle.yolox import OracleYolox, decode, two_persons
    from vge.dwpose import YOLOX_L
    fr = chain["frames"][:3]
    ob, osc = decode(OracleYolox(chain["ysd"], YOLOX_L, bf16=True).forward(fr), fr.shape[1:3], YOLOX_L.in_size)
    serr = float(np.abs(chain["cand"][:3, :, 4] - osc).max())
    print(f"detector: anchor scores max|gpu - oracle| {serr:.2e}")
    assert serr < 2e-2
    for f in range(chain["frames"].shape[0]):
        kb, n = two_persons(chain["cand"][f, :, :4], chain["cand"][f, :, 4])
        assert int(chain["npers"][f]) == n
        np.testing.assert_array_equal(chain["boxes"][f, :n], kb)


def test_crops_are_the_oracle_crops(chain):
    from oracle.hmr import vitdet_crop
    for j, f in enumerate(chain["fidx"]):
        want = vitdet_crop(chain["frames"][f], chain["gboxes"][f])
        np.testing.assert_array_equal(chain["crops"][j], want, err_msg=f"crop of frame {f}")


def test_tokenhmr_rows_vs_oracle(chain):
    from oracle.hmr import OracleHmr
    sel = [0, 1, len(chain["fidx"]) // 2, len(chain["fidx"]) - 1]
    ref = OracleHmr(chain["hsd"], chain["hcfg"], bf16=True).forward(chain["crops"][sel])
    tol = {"pose": 1.5e-2, "global_orient": 1.5e-2, "betas": 2e-2, "vit": 2e-2}   # tests/test_hmr.py
    for k, t in tol.items():
        err = float(np.abs(chain["mesh"][k][sel] - ref[k].numpy()).max())
        print(f"TokenHMR {k}: max|gpu - oracle(bf16 points)| {err:.2e}")
        assert err < t, (k, err)


def test_dwpose_rows_vs_oracle(chain):
    from oracle.dwpose import OracleRtmpose, wholebody_to_kp120
    from vge.dwpose import RTMPOSE_L as cfg
    fr, boxes, npers = chain["frames"], chain["boxes"], chain["npers"]
    H, W = fr.shape[1:3]
    inst_frame, inst_box, per_frame = [], [], []
    for f, n in enumerate(npers):   # the host's instance table: persons 0 / 1, the whole frame when nobody is found
        bl = [[0.0, 0.0, float(W), float(H)]] if n == 0 else [list(boxes[f, p]) for p in range(min(int(n), 2))]
        per_frame.append(list(range(len(inst_box), len(inst_box) + len(bl))))
        inst_frame += [f] * len(bl)
        inst_box += bl
    lv = chain["lv"]
    for f in range(fr.shape[0]):   # keypoints.npy rows = the oracle's composition of the decoded points
        ii = per_frame[f]
        want = wholebody_to_kp120(lv[ii, :, :2].numpy(), lv[ii, :, 2].numpy(), [inst_box[i] for i in ii],
                                  cfg.in_w, cfg.in_h, H, W)
        np.testing.assert_allclose(chain["rows"][f], want, rtol=0, atol=1e-6)
    sub = per_frame[0] + per_frame[T]                  # the network itself on two frames' instances
    sx, sy = OracleRtmpose(chain["psd"], cfg, bf16=True).simcc(fr, [inst_frame[i] for i in sub],
                                                               [inst_box[i] for i in sub])
    ref = torch.cat([sx, sy], -1)
    err = float((chain["simcc"][sub] - ref).abs().max())
    tol = 3e-2 * max(1.0, float(ref.abs().max()) / 4)   # tests/test_dwpose.py
    print(f"DWPose simcc: max|gpu - oracle(bf16 points)| {err:.2e} (tol {tol:.2e})")
    assert err < tol


def test_scores_of_the_extracted_files_match_the_oracle_flow(chain, tmp_path):
    """The chain's files scored by the GPU flow and by the oracle's eval.py restatement (same real set and
    checkpoint): every video scored, AC / TC within the north star's 1e-4.  The rejected clip has keypoints but no
    npz, so it is not scored (the reference's not-single list)."""
    from oracle import evalflow
    from vge import eval as VE
    from vge import synth
    paths = chain["paths"]
    got = VE.run_eval(chain["gen"], paths["real"], chain["ckpt"], chain["gkp"], paths["real_kp"], out_json=None,
                      device=DEV)
    ref, _ = evalflow.run_eval(paths["real"], paths["real_kp"], chain["gen"], chain["gkp"],
                               synth.make_state_dict(synth.DIMS_RAW, synth.DIMS_DIFF), synth.DIMS_RAW, synth.DIMS_DIFF)
    assert sorted(got) == sorted(ref) == sorted(chain["stems"][c] for c in chain["acc"])
    worst = 0.0
    for v in ref:
        assert sorted(got[v]) == sorted(ref[v]) == ["ac", "tc"]
        worst = max(worst, *(abs(got[v][k] - ref[v][k]) for k in ("ac", "tc")))
    print(f"chain scores: max|gpu - oracle| {worst:.2e} over {len(ref)} videos")
    assert worst < 1e-4
