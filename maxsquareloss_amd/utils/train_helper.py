"""get_model factory (utils/train_helper.py:9-15 of the reference)."""
from ..graphs.models.deeplab_multi import DeeplabMulti


def get_model(args):
    if args.backbone == "deeplabv2_multi":
        model = DeeplabMulti(num_classes=args.num_classes, pretrained=args.imagenet_pretrained)
        params = model.optim_parameters(args)
        args.numpy_transform = True
        return model, params
    raise ValueError(f"unsupported backbone {args.backbone!r}")
