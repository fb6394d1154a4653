"""``DataLoader`` collating :class:`Data` objects into :class:`Batch` objects.

Equivalent of ``torch_geometric.data.DataLoader(dataset, batch_size,
shuffle, follow_batch=['x_s', 'x_t'])`` used by every reference driver
(``/root/reference/examples/pascal.py:42-43``, ``willow.py:45-46``,
``pascal_pf.py:74-75``).
"""
import torch.utils.data

from .data import Batch, Data


class Collater(object):
    def __init__(self, follow_batch):
        self.follow_batch = follow_batch

    def __call__(self, batch):
        elem = batch[0]
        if isinstance(elem, Data):
            return Batch.from_data_list(batch, self.follow_batch)
        return torch.utils.data.dataloader.default_collate(batch)


class DataLoader(torch.utils.data.DataLoader):
    r"""Mini-batch loader over datasets of :class:`Data` objects."""

    def __init__(self, dataset, batch_size=1, shuffle=False, follow_batch=[],
                 **kwargs):
        kwargs.pop('collate_fn', None)
        super(DataLoader, self).__init__(
            dataset, batch_size, shuffle,
            collate_fn=Collater(follow_batch), **kwargs)
