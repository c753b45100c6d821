from .model import (INDEX_FILE_PATTERNS, build_stage, convert_to_optimized_block,  # noqa: F401
                    get_block_state_dict, get_sharded_block_state_from_file, load_block,
                    load_stage_weights, save_random_checkpoint, stage_from_hf_model)
