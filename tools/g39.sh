#!/bin/bash
# nontemporal p stores (A) / p + partial stores (B) in the tiles kernel vs the in-tree build
bash tools/ab_lib.sh A B
