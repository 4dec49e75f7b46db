// adlsm-tree_amd/csrc/rc.hpp -- return codes of the host C++ mirror.
// Same enumerators, in the same order (so the same values), as the
// reference's enum RC (src/rc.hpp:8-39); DEVICE_ERROR is new and sits after
// the reference's last code so no existing value moves.
#pragma once
#include <string_view>

namespace adl {

enum RC {
  OK,
  NOT_FOUND,
  IS_NOT_DIRECTORY,
  CREATE_DIRECTORY_FAILED,
  DESTROY_DIRECTORY_FAILED,
  DESTROY_FILE_FAILED,
  UN_IMPLEMENTED,
  EXISTED,
  OPEN_FILE_ERROR,
  IO_ERROR,
  CLOSE_FILE_ERROR,
  RENAME_FILE_ERROR,
  MAKESTEMP_ERROR,
  FILTER_BLOCK_ERROR,
  FOOTER_BLOCK_ERROR,
  UN_SUPPORTED_FORMAT,
  DB_CLOSED,
  STAT_FILE_ERROR,
  MMAP_ERROR,
  OUT_OF_RANGE,
  BAD_LEVEL,
  BAD_REVISION,
  BAD_FILE_META,
  BAD_RECORD,
  FILE_EOF,
  CHECK_SUM_ERROR,
  NOEXCEPT_SIZE,
  BAD_FILE_PATH,
  BAD_CURRENT_FILE,
  NEW_SSTABLE_ERROR,
  DEVICE_ERROR, /* new: a GPU build/probe failed (adl_status < 0 from libadlbloom) */
};

std::string_view strrc(RC rc);

}  // namespace adl
