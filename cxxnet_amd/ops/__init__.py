"""Device ops: hand-written HIP kernels on the GPU, fp32 torch reference on the CPU."""
from .gemm import (ConvGeom, conv_backward_data, conv_backward_weight, conv_forward, conv_out_size,  # noqa: F401
                   fc_backward_data, fc_backward_weight, fc_backward_weight_sgd, fc_forward)
from .nn import (act_backward, act_forward, add, copy_, bias_grad, bias_grad_multi, cast_to_bf16, channel_copy, concat_channels, dropout_apply, pad_interior, zero_, zero_ranges, fanout_copy, sum_into,  # noqa: F401
                 dropout_mask_ref, image_to_nhwc, jpeg_decode, input_to_nhwc, loss_grad, lrn_backward, lrn_backward_bias, lrn_forward, nhwc_to_nchw, pool_mask_in_state,
                 pool_backward, pool_backward_tie_all, pool_forward, pool_out_size, softmax_forward, transpose,
                 pool_lrn_forward, lrn_pool_backward, lrn_pool_backward_rows)
from .optim import fused_update, nonfinite, scale_  # noqa: F401
