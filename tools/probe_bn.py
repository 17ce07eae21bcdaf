import torch, sys
sys.path.insert(0, '/root/repo')
from semanticsegmentation_tensorflow_amd import ops
dev = torch.device("cuda:0"); BF = torch.bfloat16
for (N,H,W,C) in [(1,8,16,64),(8,384,1248,128),(2,40,52,112)]:
    for acc in (False, True):
        for s in (1, 0):
            ops.set_option("bn1x1s", s)
            d = ops.conv_desc(N, H, W, C, 64, 1, 1, dtype=ops.BF16)
            dy = torch.zeros(N,H,W,64,dtype=BF,device=dev); x = torch.zeros(N,H,W,C,dtype=BF,device=dev); dx = torch.zeros(N,H,W,C,dtype=BF,device=dev)
            wh = torch.zeros(ops.packed_shape(1,1,C,64,ops.PACK_HWIO,d.C),dtype=BF,device=dev)
            gm = torch.ones(C,device=dev); bt = torch.zeros(C,device=dev)
            rows = ops.conv_bwd_data_bn_part_rows(d)
            part = torch.empty(rows*2*d.C,device=dev)
            try:
                ops.conv2d_bwd_data_bn_part(d, dy, wh, x, gm, bt, dx, part, accumulate=acc); torch.cuda.synchronize(); r = "ok"
            except Exception as e: r = f"ERR {e}"
            print(N,H,W,C,"acc",acc,"stream",s,"rows",rows, ops.conv_kernel_info(d, ops.OP_BWD_DATA_BN)[0], r, flush=True)
ops.set_option("bn1x1s", 1)
