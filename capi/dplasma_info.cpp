// dplasma_info_t: the string key/value option object of the reference (src/utils/dplasma_info.{h,c},
// src/utils/dplasma_info.c:43-152), native in the C ABI (no interpreter involved).  Keys keep their
// first-insertion order; setting an existing key replaces its value; get_nthkey indexes that order.
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "capi_bridge.h"

#define DPLASMA_MAX_INFO_KEY 255
#define DPLASMA_MAX_INFO_VAL 1024

struct dplasma_info_s {
  std::vector<std::pair<std::string, std::string>> kv;
};
typedef struct dplasma_info_s* dplasma_info_t;

static std::vector<std::pair<std::string, std::string>>::iterator find_key(dplasma_info_t info, const char* key) {
  auto it = info->kv.begin();
  for (; it != info->kv.end(); ++it)
    if (it->first == key) break;
  return it;
}

extern "C" {

DPL_CAPI int dplasma_info_create(dplasma_info_t* info) {
  if (!info) return -1;
  *info = new dplasma_info_s;
  return 0;
}

DPL_CAPI int dplasma_info_free(dplasma_info_t* info) {
  if (!info || !*info) return -1;
  delete *info;
  *info = nullptr;
  return 0;
}

DPL_CAPI int dplasma_info_set(dplasma_info_t info, const char* key, const char* value) {
  if (!info || !key || !value || std::strlen(key) > DPLASMA_MAX_INFO_KEY || std::strlen(value) > DPLASMA_MAX_INFO_VAL)
    return -1;
  auto it = find_key(info, key);
  if (it != info->kv.end()) it->second = value;
  else info->kv.emplace_back(key, value);
  return 0;
}

DPL_CAPI int dplasma_info_delete(dplasma_info_t info, const char* key) {
  if (!info || !key) return -1;
  auto it = find_key(info, key);
  if (it == info->kv.end()) return -1;
  info->kv.erase(it);
  return 0;
}

DPL_CAPI int dplasma_info_get(dplasma_info_t info, const char* key, int valuelen, char* value, int* flag) {
  if (flag) *flag = 0;
  if (!info || !key) return -1;
  auto it = find_key(info, key);
  if (it == info->kv.end()) return 0;
  if (flag) *flag = 1;
  if (value && valuelen > 0) {
    std::strncpy(value, it->second.c_str(), (size_t)valuelen - 1);
    value[valuelen - 1] = '\0';
  }
  return 0;
}

DPL_CAPI int dplasma_info_get_nkeys(dplasma_info_t info, int* nkeys) {
  if (!info || !nkeys) return -1;
  *nkeys = (int)info->kv.size();
  return 0;
}

DPL_CAPI int dplasma_info_get_nthkey(dplasma_info_t info, int n, char* key) {
  if (!info || !key || n < 0 || n >= (int)info->kv.size()) return -1;
  std::strncpy(key, info->kv[(size_t)n].first.c_str(), DPLASMA_MAX_INFO_KEY);
  key[DPLASMA_MAX_INFO_KEY] = '\0';
  return 0;
}

}  // extern "C"
