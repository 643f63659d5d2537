/*
 * swim.h — C ABI of the lockstep SWIM simulation engine (libswimgpu.so).
 *
 * One engine handle simulates N virtual scalecube-cluster members in lockstep virtual time.
 * It replaces, for all N members at once, the three protocol objects that
 * ClusterImpl.doStart0 constructs (cluster/src/main/java/io/scalecube/cluster/ClusterImpl.java:260-291):
 *   FailureDetectorImpl   (cluster/.../fdetector/FailureDetectorImpl.java:75-99)
 *   GossipProtocolImpl    (cluster/.../gossip/GossipProtocolImpl.java:81-104)
 *   MembershipProtocolImpl(cluster/.../membership/MembershipProtocolImpl.java:120-168)
 * plus the Transport + NetworkEmulator underneath them
 * (cluster-testlib/.../utils/NetworkEmulatorTransport.java:49-83, NetworkEmulator.java:167-202,349-369).
 *
 * Plain C: integers, pointers and sizes only.  Every function returns an int32 status
 * (SWIM_OK or a negative SWIM_E* code); nothing throws across the ABI.  A handle is
 * single-threaded, mirroring the reference's one-scheduler-per-member confinement
 * (ClusterImpl.java:257).  The engine owns all device memory; callers own output buffers.
 *
 * The same ABI is exported by the CPU oracle (oracle/liboracle_swim.so, test infrastructure
 * only) so that parity tests drive both through identical code.
 */
#ifndef SWIM_H
#define SWIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------------------ */
#define SWIM_OK 0
#define SWIM_EINVAL (-1)     /* bad argument / unsupported configuration */
#define SWIM_ENOMEM (-2)     /* device or host allocation failed */
#define SWIM_EDEVICE (-3)    /* HIP runtime error or no MI355X device */
#define SWIM_ECAPACITY (-4)  /* a fixed-capacity structure overflowed; state is no longer exact */
#define SWIM_ESTATE (-5)     /* operation not valid in the member's current state */

/* ---- member status (MemberStatus.java:3-19, declaration order) ------------------------ */
#define SWIM_ALIVE 0
#define SWIM_SUSPECT 1
#define SWIM_LEAVING 2
#define SWIM_DEAD 3

/* ---- membership event types (MembershipEvent.java:15-20, declaration order) ----------- */
#define SWIM_EV_ADDED 0
#define SWIM_EV_REMOVED 1
#define SWIM_EV_LEAVING 2
#define SWIM_EV_UPDATED 3
/* FailureDetectorEvent (FailureDetectorEvent.java:8-33), only when record_fd_events = 1 */
#define SWIM_EV_FD_ALIVE 16
#define SWIM_EV_FD_SUSPECT 17
#define SWIM_EV_FD_DEAD 18
/* user gossips (GossipProtocol.spread / listen, GossipProtocolImpl.java:126-130,201-215,167-180):
 * GOSSIP: viewer received a new user gossip (listen() emits it); subject = its gossiper, data = payload.
 * SPREAD_DONE: the spread() Mono of viewer's own gossip completed (the first gossip round with
 * period > infectionPeriod + periodsToSpread); subject = viewer, data = payload. */
#define SWIM_EV_GOSSIP 32
#define SWIM_EV_SPREAD_DONE 33
/* swim_gossip.status of a user gossip (its subject field holds the payload): USER until the
 * originator's spread() completes, USER_SPREAD afterwards (copies sent from then on carry it too) */
#define SWIM_GOSSIP_USER 4
#define SWIM_GOSSIP_USER_SPREAD 5

/* ---- canonical intra-tick phases ---------------------------------------- */
#define SWIM_PHASE_TIMERS 1  /* suspicion timeouts      (MembershipProtocolImpl.java:825-834) */
#define SWIM_PHASE_FD 2      /* ping / ping-req / ack    (FailureDetectorImpl.java:126-210)   */
#define SWIM_PHASE_GOSSIP 3  /* one gossip round         (GossipProtocolImpl.java:141-215)    */
#define SWIM_PHASE_SYNC 4    /* SYNC requests delivered  (MembershipProtocolImpl.java:394-415)*/
#define SWIM_PHASE_SYNCACK 5 /* SYNC_ACKs delivered      (MembershipProtocolImpl.java:385-391)*/
#define SWIM_PHASE_CONTROL 6 /* host control ops (leave, join) applied between ticks          */
#define SWIM_PHASE_FETCH 7   /* delayed GET_METADATA round trips arriving (MetadataStoreImpl.java:146-185),
                                processed first in the tick; events sort by (tick, viewer, phase, minor) */

/*
 * Packed view cell: one 64-bit word per (viewer, subject).  This is also the readback format of
 * swim_read_view.  It holds the viewer's MembershipRecord for the subject
 * (MembershipRecord.java:20-22) plus the per-subject bits the reference keeps in side maps:
 * `members` (MembershipProtocolImpl.java:89), `aliveEmittedSet` (:91), the MetadataStore entry
 * (MetadataStoreImpl.java:104-143) and the suspicion task (:105, :805-823).
 *   bits  0..31  incarnation (int32, MembershipRecord.java:22)
 *   bits 32..33  status (SWIM_ALIVE / SWIM_SUSPECT / SWIM_LEAVING; DEAD is never stored)
 *   bit  34      in_table       — row present in membershipTable
 *   bit  35      in_members     — subject present in the `members` map
 *   bit  36      alive_emitted  — subject present in aliveEmittedSet
 *   bit  37      has_timer      — a suspicion timeout task is scheduled
 *   bit  38      has_metadata   — MetadataStore holds metadata for the subject
 *   bits 39..63  timer deadline tick (mod 2^25), valid when has_timer
 */
#define SWIM_CELL_INC(c) ((int32_t)(uint32_t)((c)&0xffffffffull))
#define SWIM_CELL_STATUS(c) ((uint32_t)(((c) >> 32) & 3u))
#define SWIM_CELL_IN_TABLE(c) ((uint32_t)(((c) >> 34) & 1u))
#define SWIM_CELL_IN_MEMBERS(c) ((uint32_t)(((c) >> 35) & 1u))
#define SWIM_CELL_ALIVE_EMITTED(c) ((uint32_t)(((c) >> 36) & 1u))
#define SWIM_CELL_HAS_TIMER(c) ((uint32_t)(((c) >> 37) & 1u))
#define SWIM_CELL_HAS_METADATA(c) ((uint32_t)(((c) >> 38) & 1u))
#define SWIM_CELL_DEADLINE(c) ((uint32_t)((c) >> 39))
#define SWIM_DEADLINE_MASK 0x1ffffffu

/*
 * Protocol configuration.  Field-for-field mirror of the reference knobs
 * (FailureDetectorConfig.java:9-25, GossipConfig.java:9-25, MembershipConfig.java:14-32,
 * ClusterConfig.java:28-38) plus engine knobs.  All times are milliseconds of virtual time.
 */
typedef struct swim_config {
  /* FailureDetectorConfig */
  int32_t ping_interval;      /* DEFAULT_PING_INTERVAL = 1000 */
  int32_t ping_timeout;       /* DEFAULT_PING_TIMEOUT = 500 (must be < ping_interval) */
  int32_t ping_req_members;   /* DEFAULT_PING_REQ_MEMBERS = 3 (<= 16) */
  /* GossipConfig */
  int32_t gossip_interval;    /* DEFAULT_GOSSIP_INTERVAL = 200 */
  int32_t gossip_fanout;      /* DEFAULT_GOSSIP_FANOUT = 3 (<= 16) */
  int32_t gossip_repeat_mult; /* DEFAULT_GOSSIP_REPEAT_MULT = 3 */
  int32_t gossip_segmentation_threshold; /* GOSSIP_SEGMENTATION_THRESHOLD = 1000 */
  /* MembershipConfig */
  int32_t sync_interval;      /* DEFAULT_SYNC_INTERVAL = 30000 */
  int32_t sync_timeout;       /* DEFAULT_SYNC_TIMEOUT = 3000 */
  int32_t suspicion_mult;     /* DEFAULT_SUSPICION_MULT = 5 */
  int32_t removed_members_history_size; /* 42 (monitoring only; kept for config fidelity) */
  /* ClusterConfig */
  int32_t metadata_timeout;   /* DEFAULT_METADATA_TIMEOUT = 3000 */
  /* ---- engine knobs (no reference counterpart) ---- */
  int32_t tick_ms;            /* 0 = gcd of every interval/timeout above */
  int32_t sync_stagger;       /* 1 = each initial member's periodic SYNC gets a random phase */
  int32_t record_fd_events;   /* 1 = FailureDetectorEvents appear in the event stream */
  uint32_t gossip_capacity;   /* max live GossipStates per member (0 = default 1024; a member keeps
                                 every gossip of the last 2 x (spread + 1) rounds, so churn needs more) */
  uint32_t collector_capacity;/* hash slots for the SequenceIdCollectors a member holds, one per
                                 distinct gossiper heard (power of two; 0 = default 4096; keep the
                                 load well below 1: open addressing) */
  uint32_t event_capacity;    /* undrained events the engine may buffer (0 = default 1<<22) */
  int32_t device;             /* HIP device ordinal the engine runs on (one engine per GPU) */
  int32_t local_shards;       /* swim_create only: > 1 runs the cluster as this many row shards in
                                 one process on `device`, exchanging cross-shard messages with
                                 device copies (the single-GPU test rig of swim_create_shard) */
  int32_t timer_stagger;      /* 1 = each initial member's ping and gossip timers also get a random
                                 phase (members of a real cluster start at different instants; the
                                 default 0 aligns them) */
  uint32_t timer_capacity;    /* suspicion timers that may fall due in one tick, per row shard, split
                                 over the shard's 256-viewer blocks (2x the even share, at least 4,096 each)
                                 (0 = default 2 x the shard's rows; churn schedules a timer for every
                                 killed member at every viewer within a few seconds) */
  uint32_t message_capacity;  /* GOSSIP_REQ messages one gossip round may materialise, per row shard
                                 (0 = default 512 x the shard's rows; loss and churn storms need more) */
  uint32_t interval_capacity; /* spilled SequenceIdCollector blocks per row in the smallest size tier
                                 (0 = default 64; the larger tiers scale with it): collectors with
                                 many gaps (lossy links drop gossips) spill out of their inline entry */
  uint32_t deliver_wave_min;  /* gossip inboxes above this many messages are delivered by a whole wave
                                 (0 = default 24, the most the per-thread LDS sort holds; a test knob:
                                 1 sends every inbox through the wave path) */
  uint32_t delay_capacity;    /* delayed GOSSIP_REQs that may arrive in one tick (0 = default 1,024;
                                 allocated when a message delay is first set) */
  uint32_t timer_pool_capacity; /* suspicion timers pending at once, per row shard, over all deadlines
                                 (0 = default: the wheel's deadline buckets x timer_capacity, capped
                                 at 2^27; a 2-way partition holds N/2 timers at every viewer) */
} swim_config;

/* preset: 0 = defaultConfig/defaultLanConfig, 1 = defaultWanConfig, 2 = defaultLocalConfig
 * (ClusterConfig.java:54-93) */
int32_t swim_config_default(swim_config* cfg, int32_t preset);

/* ClusterMath (ClusterMath.java:38-135) */
int32_t swim_ceil_log2(int32_t num);                                       /* :133-135 */
int32_t swim_gossip_periods_to_spread(int32_t repeat_mult, int32_t cluster_size); /* :111-113 */
int32_t swim_gossip_periods_to_sweep(int32_t repeat_mult, int32_t cluster_size);  /* :99-102 */
int64_t swim_suspicion_timeout(int32_t suspicion_mult, int32_t cluster_size,
                               int64_t ping_interval);                      /* :123-125 */

typedef struct swim_engine swim_engine;

/*
 * Create an engine with `capacity` member slots (slot = member address; member ids are slot
 * numbers).  Slots [0, n_initial) start up and fully converged: every table holds every initial
 * member ALIVE at incarnation 0 and every ping / gossip list is a seeded shuffle.  Slots
 * [n_initial, capacity) are free until swim_join.  `seed` keys the counter-based Philox RNG that
 * replaces ThreadLocalRandom / Collections.shuffle.
 */
int32_t swim_create(const swim_config* cfg, uint32_t capacity, uint32_t n_initial, uint64_t seed,
                    swim_engine** out);
int32_t swim_destroy(swim_engine* e);

/*
 * Multi-GPU: one process per GPU, member rows sharded by viewer.  Rank r of `world`
 * owns viewers [r*ceil(N/world), (r+1)*ceil(N/world)); GOSSIP_REQ, SYNC and SYNC_ACK traffic to
 * other shards moves by RCCL send/recv over xGMI inside swim_step.  Rank 0 calls
 * swim_comm_unique_id and the host broadcasts the SWIM_COMM_ID_BYTES bytes to every rank (the
 * reference has no counterpart: its members are separate JVM objects talking over TCP,
 * ClusterImpl.java:260-291 + TransportImpl.java:214-238).  Every swim_* call on a sharded engine is
 * collective: all ranks make the same calls in the same order (control ops are replicated, reads of
 * rows / members / lists / gossips / collectors are answered only by the owning rank and return
 * SWIM_EINVAL elsewhere; events and stats are those of the rank's own viewers).
 */
#define SWIM_COMM_ID_BYTES 128
int32_t swim_comm_unique_id(uint8_t* out /* SWIM_COMM_ID_BYTES */);
int32_t swim_create_shard(const swim_config* cfg, uint32_t capacity, uint32_t n_initial, uint64_t seed,
                          int32_t rank, int32_t world, const uint8_t* comm_id, swim_engine** out);
/* rank / world of the engine and the viewer range [lo, lo + count) it answers reads for */
int32_t swim_shard_info(const swim_engine* e, int32_t* rank, int32_t* world, uint32_t* lo, uint32_t* count);
/*
 * swim_create_shard with world = 1 and a comm_id is an RCCL engine of ONE rank: the whole exchange
 * machinery runs (count all-to-alls, the IPC handle of its own exchange region and its all-gather,
 * the row pulls, the quiet windows' allreduces) with nothing to exchange — the transport on one GPU.
 * swim_exchange_info reports how the exchange is set up (no reference counterpart):
 */
#define SWIM_XCHG_ON 1u            /* sharded tick path with exchange kernels (world > 1 or RCCL) */
#define SWIM_XCHG_RCCL 2u          /* RCCL transport (one process per GPU) */
#define SWIM_XCHG_UNCACHED 4u      /* the exchange region is uncached device memory */
#define SWIM_XCHG_IPC 8u           /* an IPC handle of the region was exported to the peers */
#define SWIM_XCHG_IPC_FALLBACK 16u /* the uncached region had no IPC handle: re-allocated cached */
int32_t swim_exchange_info(const swim_engine* e, uint32_t* flags);

/* Advance virtual time.  swim_step advances `periods` * (ping_interval / tick) ticks. */
int32_t swim_step_ticks(swim_engine* e, uint32_t ticks);
int32_t swim_step(swim_engine* e, uint32_t periods);
int32_t swim_now(const swim_engine* e, uint64_t* tick, uint32_t* tick_ms, uint32_t* ticks_per_period);

/* ---- seeds (MembershipConfig.seedMembers, MembershipProtocolImpl.java:143,461-472) ------ */
/* The seed list of every member that has no list of its own (duplicates dropped in order, as
 * cleanUpSeedMembers' LinkedHashSet does, :171-190). */
int32_t swim_set_seeds(swim_engine* e, const uint32_t* seeds, uint32_t n_seeds);
/* Member m's own MembershipConfig.seedMembers (each member's ClusterConfig, MembershipProtocolImpl
 * constructor :120-130 -> cleanUpSeedMembers :171-190; SimulatedCluster maps one config per member):
 * duplicates dropped in order; from the next step on, m's start0 sends its initial SYNCs to these
 * (:250-291) and its selectSyncAddress draws from them U otherMembers (:461-472) instead of the
 * engine-wide list.  n_seeds = 0 gives m an empty list; seeds = NULL with n_seeds = UINT32_MAX puts m
 * back on the engine-wide list.  Replicated: every rank of a sharded engine makes the same call. */
int32_t swim_set_member_seeds(swim_engine* e, uint32_t m, const uint32_t* seeds, uint32_t n_seeds);

/* ---- lifecycle --------------------------------------------------------------------------- */
/* Stop member m's transport abruptly (TransportImpl.stop): sends to it fail at the sender. */
int32_t swim_kill(swim_engine* e, uint32_t m);
/* Graceful shutdown (ClusterImpl.doShutdown :508-517): LEAVING inc+1 gossip now
 * (MembershipProtocolImpl.leaveCluster :233-242); the member stops once that gossip's spread()
 * completes (GossipProtocolImpl.java:167-180). stop_after = 0 only publishes LEAVING. */
int32_t swim_leave(swim_engine* e, uint32_t m, int32_t stop_after);
/* Start a fresh member in free slot m (ClusterImpl.doStart0 + MembershipProtocolImpl.start0
 * :250-291): initial SYNC to every seed during the next tick. */
int32_t swim_join(swim_engine* e, uint32_t m);
/* swim_join, with member m's transport bound to the address of member addr_of, whose transport is
 * stopped: a restart on the same port (MembershipProtocolTest.testRestartStoppedMembersOnSameAddresses
 * :654-711).  From m's start on, every message sent to addr_of's address reaches m:
 *   - its onPing answers DEST_GONE (FailureDetectorImpl.onPing :227-259), which the pinger's
 *     computeMemberStatus turns into DEAD (:382-404), directly or through a relay (:291-315);
 *   - a GET_METADATA request for addr_of goes unanswered (MetadataStoreImpl.onMetadataRequest :209);
 *   - gossips and SYNCs to addr_of are delivered to m;
 * and m ignores records of other members at its own address (MembershipProtocolImpl.updateMembership
 * :605-610) and drops that address from its seeds (cleanUpSeedMembers :171-190).
 * SWIM_ESTATE if the address is in use (its holder is up or about to start). */
int32_t swim_join_at(swim_engine* e, uint32_t m, uint32_t addr_of);
/* GossipProtocol.spread(Message) (GossipProtocolImpl.java:126-130 -> createAndPutGossip :190-199)
 * on member m now, between ticks: a user gossip carrying the 32-bit payload (a handle the caller
 * maps to the message).  Receivers report it with SWIM_EV_GOSSIP, the originator's spread()
 * completion with SWIM_EV_SPREAD_DONE. */
int32_t swim_spread(swim_engine* e, uint32_t m, uint32_t payload);

/* ClusterImpl.updateMetadata (:497-500): member m's metadata changes (its version + 1) and
 * MembershipProtocolImpl.updateIncarnation (:214-226) puts ALIVE inc+1 and spreads it; a viewer
 * that then admits the record fetches the new metadata and publishes UPDATED (:780-781). */
int32_t swim_update_metadata(swim_engine* e, uint32_t m);
/* MembershipConfig.namespace of every member as a group id (ns_of_member[capacity] < n_ns) and the
 * n_ns x n_ns matrix related[a * n_ns + b] = areNamespacesRelated(a, b) (:511-536): updateMembership
 * skips records of members in unrelated namespaces (:575-586).  n_ns = 0 restores one namespace.
 * SWIM_ESTATE if two initially joined members are unrelated (the converged start holds both). */
int32_t swim_set_namespaces(swim_engine* e, const uint16_t* ns_of_member, uint32_t n_ns, const uint8_t* related);

/* ---- network emulator (NetworkEmulator.java) ----------------------------------------------
 * Outbound loss is decided at the sender and fails the send immediately (:167-181); inbound
 * blocking silently drops at the receiver (NetworkEmulatorTransport.java:69-83). */
/* setDefaultOutboundSettings(lossPercent, 0) (:80-83); m = UINT32_MAX applies to every member */
int32_t swim_set_default_loss(swim_engine* e, uint32_t m, int32_t loss_percent);
/* outboundSettings(dst, loss, 0) on src (:69-73); loss_percent < 0 removes the override
 * (unblockOutbound :134-139) */
int32_t swim_set_link_loss(swim_engine* e, uint32_t src, uint32_t dst, int32_t loss_percent);
/* The meanDelay half of setDefaultOutboundSettings(loss, meanDelay) (:80-83) and of
 * outboundSettings(dst, loss, meanDelay) on src (:69-73); mean_ms < 0 removes the link override.
 * A message is delivered floor(delay / tick_ms) ticks after it was sent, delay drawn as
 * evaluateDelay (:359-369) from the Philox hook (swim_delay.h).  Applies to the failure
 * detector's pings, ping-reqs and acks (a round trip completes when both legs arrived; a late
 * direct ack joins the ping-req race, :153-210) and to GOSSIP_REQs (delivered in the gossip phase
 * of their arrival tick, after the arrivals of earlier rounds), to SYNC / SYNC_ACK (each delayed
 * message carries its content as prepared; start0's initial-sync timeout restarts at every
 * answer, MembershipProtocolImpl.java:268-289) and to GET_METADATA round trips (a fetch whose round
 * trip reaches metadataTimeout fails, MetadataStoreImpl.java:146-185); DESIGN.md §3.  Sharded
 * engines too (a delayed message waits in its sender's shard and joins the exchange of its
 * arrival tick); N <= 2^20 (SWIM_EINVAL otherwise).
 * A mean above SWIM_DELAY_MEAN_MAX_TICKS (64) ticks is refused with SWIM_EINVAL: the quantised
 * delay is capped at SWIM_DELAY_TICKS_MAX ticks and would truncate draws (swim_delay.h). */
int32_t swim_set_default_delay(swim_engine* e, uint32_t m, int32_t mean_ms);
int32_t swim_set_link_delay(swim_engine* e, uint32_t src, uint32_t dst, int32_t mean_ms);
/* inboundSettings(src, shallPass) on dst (:219-223); shall_pass < 0 removes the override */
int32_t swim_set_link_inbound(swim_engine* e, uint32_t dst, uint32_t src, int32_t shall_pass);
/* setDefaultInboundSettings(shallPass) (:230-233); m = UINT32_MAX applies to every member */
int32_t swim_set_default_inbound(swim_engine* e, uint32_t m, int32_t shall_pass);
/* Partition shorthand: outbound between members of different groups is blocked (100 % loss at
 * the sender, NetworkEmulator.blockOutbound :117-121).  groups = NULL heals the partition. */
int32_t swim_set_partition(swim_engine* e, const uint16_t* group_of_member);

/* ---- readback --------------------------------------------------------------------------- */
/* Viewer's whole row, `capacity` packed cells (format above). */
int32_t swim_read_view(swim_engine* e, uint32_t viewer, uint64_t* out_cells);

typedef struct swim_event {
  uint64_t tick;
  uint32_t viewer;
  uint32_t subject;
  uint32_t type;  /* SWIM_EV_* */
  uint32_t phase; /* SWIM_PHASE_* */
  uint32_t minor; /* order within (tick, viewer, phase) */
  uint32_t data;  /* SWIM_EV_GOSSIP / SWIM_EV_SPREAD_DONE: the payload; 0 otherwise */
} swim_event;
/* Events in canonical order (tick, viewer, phase, minor).  *n_out = events copied; events that
 * did not fit stay buffered for the next call. */
int32_t swim_drain_events(swim_engine* e, swim_event* out, size_t cap, size_t* n_out);

typedef struct swim_stats {
  uint64_t ticks;
  uint64_t pings;             /* doPing with a target            */
  uint64_t ping_reqs;         /* doPingReq launches              */
  uint64_t fd_events;         /* FailureDetectorEvents published */
  uint64_t gossips_created;   /* createAndPutGossip              */
  uint64_t gossip_messages;   /* GOSSIP_REQ messages sent        */
  uint64_t gossip_accepted;   /* first receipts (collector add)  */
  uint64_t syncs;             /* SYNC messages sent              */
  uint64_t sync_acks;         /* SYNC_ACK messages delivered     */
  uint64_t sync_records;      /* records merged by syncMembership */
  uint64_t fetches;           /* GET_METADATA round trips issued */
  uint64_t fetch_ok;
  uint64_t timers_fired;
  uint64_t events;
  uint64_t capacity_errors;
  /* gossips_created split by the reference call site that originated each gossip (SWIM_ORIG_*) */
  uint64_t gossips_by_reason[7];
  uint64_t reserved[2];
} swim_stats;
/* Gossip origination reasons (the callers of spreadMembershipGossip / GossipProtocol.spread in
 * MembershipProtocolImpl.java; MEMBERSHIP_GOSSIP and INITIAL_SYNC never originate, :836-843):
 *   FD       SUSPECT from a FailureDetector event          (updateMembership :621-628, reason FD)
 *   SYNC     SUSPECT or admitted ALIVE learned from a SYNC / SYNC_ACK   (:621-628, :648-656)
 *   REFUTE   ALIVE/LEAVING inc+1 about oneself              (onSelfMemberDetected :686-708)
 *   LEAVING  a received LEAVING record re-spread            (onLeavingDetected :710-733)
 *   LEAVE    own graceful leave                             (leaveCluster :233-242)
 *   METADATA own metadata update                            (updateIncarnation :214-226)
 *   USER     GossipProtocol.spread                          (GossipProtocolImpl.java:126-130) */
#define SWIM_ORIG_FD 0
#define SWIM_ORIG_SYNC 1
#define SWIM_ORIG_REFUTE 2
#define SWIM_ORIG_LEAVING 3
#define SWIM_ORIG_LEAVE 4
#define SWIM_ORIG_METADATA 5
#define SWIM_ORIG_USER 6
int32_t swim_get_stats(swim_engine* e, swim_stats* out);

/* ---- full-state readback for parity tests (not needed by a Java host) --------------------- */
typedef struct swim_member_state {
  uint8_t up;
  uint8_t joined;
  uint8_t leave_pending;     /* graceful leave waiting for its gossip to spread */
  uint8_t join_pending;      /* initial sync scheduled for the next tick */
  int32_t remote_idx;        /* GossipProtocolImpl.remoteMembersIndex */
  uint64_t fd_period;        /* FailureDetectorImpl.currentPeriod */
  uint32_t ping_cursor;      /* FailureDetectorImpl.pingMemberIndex */
  uint32_t ping_len;
  uint32_t remote_len;
  uint32_t gossip_len;       /* live GossipStates */
  uint64_t gossip_period;    /* GossipProtocolImpl.currentPeriod */
  uint64_t gossip_counter;   /* GossipProtocolImpl.gossipCounter */
  uint32_t table_size;       /* membershipTable.size() */
  uint32_t members_size;     /* members.size() */
  int64_t fd_start, gossip_start, sync_start; /* timer phases (ticks); sync_start valid if sync_on */
  uint8_t sync_on;
  uint8_t pad[3];
  uint32_t ack_target;       /* pending ping-req launch (ack timeout) */
  uint64_t ack_due;          /* 0 = none */
  uint32_t relay_target;     /* pending relay timeouts */
  uint32_t relay_pending;
  uint64_t relay_due;        /* 0 = none */
  uint32_t leave_gossiper;   /* id of the LEAVING gossip a graceful leave waits on */
  uint32_t pending_acks;     /* merged SYNCs whose SYNC_ACK waits for their updateMembership Monos
                                (onSync :394-415) + start0 groups its doFinally waits for (:277-289) */
  uint64_t leave_seq;
} swim_member_state;
int32_t swim_read_member(swim_engine* e, uint32_t m, swim_member_state* out);
/* FailureDetectorImpl.pingMembers / GossipProtocolImpl.remoteMembers in list order */
int32_t swim_read_ping_list(swim_engine* e, uint32_t m, uint32_t* out, uint32_t cap, uint32_t* len);
int32_t swim_read_remote_list(swim_engine* e, uint32_t m, uint32_t* out, uint32_t cap, uint32_t* len);

typedef struct swim_gossip {
  uint32_t gossiper;          /* Gossip.gossiperId */
  uint32_t subject;           /* MembershipRecord carried as the gossip payload */
  uint64_t seq;               /* Gossip.sequenceId */
  int32_t inc;
  uint32_t status;
  uint64_t infection_period;  /* GossipState.infectionPeriod */
  uint32_t infected[2];       /* GossipState.infected (UINT32_MAX = empty slot) */
} swim_gossip;
/* Live gossips of member m in canonical (insertion) order. */
int32_t swim_read_gossips(swim_engine* e, uint32_t m, swim_gossip* out, uint32_t cap, uint32_t* len);

typedef struct swim_interval {
  uint64_t lo, hi;
} swim_interval;
/* SequenceIdCollector of (m, gossiper): closed intervals in ascending order. */
int32_t swim_read_collector(swim_engine* e, uint32_t m, uint32_t gossiper, swim_interval* out,
                            uint32_t cap, uint32_t* len);

/* ---- measurement ---------------------------------------------------------------------------
 * Per-kernel timing of the SYNC classification kernel (k_sync_classify, the SYNC row stream: it
 * classifies every SYNC and, from the same loads, the SYNC_ACK answering it), measured with HIP
 * events bound to one launch in three on the engine's own stream.  For those sampled launches:
 * `launches`, `total_ms`, `messages` / `records` they processed, and `alg_bytes`: per streamed
 * (message, 1,024-subject block) unit the record words of the content row and of the receiver row
 * (2 x 1,024 x 4 B), 8 B per unit skipped by the exact block witness (its two block counts), plus
 * 4 B per record routed to the sequential merge.  enable = 0 stops recording; enable = 1
 * (re)starts it from zero.  The CPU oracle reports zeros. */
typedef struct swim_kernel_profile {
  uint64_t launches;
  double total_ms;
  uint64_t messages;   /* merge: (SYNC, 1,024-subject block) units whose two rows were streamed;
                          fanout: GOSSIP_REQs materialised */
  uint64_t records;    /* records that changed a table (sequential merge path) */
  uint64_t alg_bytes;
  uint64_t examined;   /* fanout: the states whose 16 hot bytes the rounds read (swept prefix + the
                          passes over the in-window suffix), of the `records` live ones */
} swim_kernel_profile;
int32_t swim_profile_enable(swim_engine* e, int32_t enable);
int32_t swim_profile_merge(swim_engine* e, swim_kernel_profile* out);
/* The gossip fanout kernel (doSpreadGossip's sends, k_gossip_emit), sampled the same way:
 * messages = GOSSIP_REQs materialised, records = (gossip, sender round) states read,
 * alg_bytes = 24 B x messages + 32 B x records (SURVEY.md §8(d) fanout). */
int32_t swim_profile_fanout(swim_engine* e, swim_kernel_profile* out);
/* The gossip delivery kernel (onGossipReq for every inbox, k_gossip_deliver), sampled the same way:
 * messages = GOSSIP_REQs delivered, records = those accepted (new GossipStates), alg_bytes =
 * 24 B x messages + 24 B (8 B dedupe RMW + 16 B view RMW) x messages not flagged as provable
 * duplicates by the sender (SURVEY.md §8(d) merge). */
int32_t swim_profile_deliver(swim_engine* e, swim_kernel_profile* out);

/* ---- external SYNC ingestion (parity with a JVM unpinned) ---------------
 * onSyncAck for a SYNC / SYNC_ACK that arrived from outside the simulation, e.g. decoded with
 * swimgpu.wire from a real JVM node's bytes (MembershipProtocolImpl.java:363-391): syncMembership
 * (:491-509) at viewer v over n records — member slot, status (SWIM_ALIVE / SWIM_SUSPECT / SWIM_LEAVING),
 * incarnation — in the given order, reason SYNC (initial = 0) or INITIAL_SYNC, applied between ticks
 * at the current tick with phase SWIM_PHASE_CONTROL: every updateMembership branch (namespace filter,
 * isOverrides, refutation, LEAVING, SUSPECT timers, ALIVE admissions through the metadata round trip),
 * gossip origination, events, ping / remote list updates.  Counted as one SYNC_ACK carrying n
 * records.  SWIM_EINVAL for n > members, a member out of range, a negative incarnation or a DEAD
 * record (a SyncData never holds one: the table drops DEAD members, :617-618 / onDeadMemberDetected);
 * SWIM_ESTATE if v is not running; sharded: the owning rank applies it. */
typedef struct swim_record {
  uint32_t member;
  uint32_t status;
  int32_t inc;
  uint32_t pad;
} swim_record;
int32_t swim_ingest_sync(swim_engine* e, uint32_t viewer, const swim_record* records, uint32_t n, int32_t initial);

/* ---- quiet windows ---------------------------------------------------------
 * While the cluster is provably quiet — no live gossip, no pending failure-detector or suspicion
 * work, every up member's table equal to the reference row with no SUSPECT / LEAVING record, no loss,
 * per-link setting, partition, delay, address route or control operation pending — every tick is
 * member-local (each ping acknowledged at once, gossip rounds with nothing to send,
 * MembershipProtocolImpl.doSync merging identical tables), and swim_step_ticks advances a whole
 * window of ticks with two kernel launches, the window ending at the first tick that needs the
 * per-tick kernel chain.  Results are identical either way.  enable = 0 forces the per-tick chain
 * (A/B measurement, tests); the default is on (SWIM_QUIET=0 in the environment at creation turns it
 * off).  The CPU oracle accepts the call and ignores it. */
int32_t swim_set_quiet_path(swim_engine* e, int32_t enable);
typedef struct swim_quiet_stats {
  uint64_t ticks;      /* ticks advanced inside quiet windows */
  uint64_t windows;    /* windows that advanced at least one tick */
  uint64_t attempts;   /* windows tried (a scan that found the cluster not quiet advances none) */
  uint64_t cut_short;  /* windows that ended before their length at a tick needing the per-tick chain */
  uint64_t precomputed; /* windows whose end the previous window's apply had found (no scan launch) */
} swim_quiet_stats;
int32_t swim_get_quiet_stats(const swim_engine* e, swim_quiet_stats* out);
/* The quiet windows' kernels (k_quiet_scan .. k_quiet_apply of one window, HIP events on the engine's
 * stream), every window while profiling is enabled (swim_profile_enable): launches = windows,
 * messages = ticks advanced, records = member-periods advanced (rows x ticks / ticks per period),
 * alg_bytes = 21 B per member-period (SURVEY.md §8(d) ping phase: list word, cursor, up word, view
 * word) + per window what the quiet check reads: the 4-B count of non-zero witness blocks and 64 B
 * of member words per row, the reference row (4 B per subject per shard), 4 B per timer-bucket queue of the
 * window.  The CPU oracle reports zeros. */
int32_t swim_profile_quiet(swim_engine* e, swim_kernel_profile* out);

/* Profiling builds (-DSWIM_PHASE_PROF, tools/phase_prof.sh) only: per-phase wall-time sums of the
 * instrumented kernels (100 MHz ticks), n <= 64 slots; reset = 1 zeroes them.  The product build and
 * the CPU oracle report zeros. */
int32_t swim_debug_counters(uint64_t* out, uint32_t n, int32_t reset);

/* ---- known-answer hooks (run the engine's own merge / dedupe code on given inputs) --------- */
/* Philox4x32-10 block used by every draw site. */
int32_t swim_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
/* MembershipRecord.isOverrides for n cases; case i = cases[5i..5i+4] =
 * {r1_status, r1_inc, r0_present, r0_status, r0_inc}; out[i] = 0/1 (MembershipRecordTest). */
int32_t swim_kat_overrides(const int32_t* cases, uint32_t n, uint8_t* out);
/* One SequenceIdCollector driven by n ops (SequenceIdCollectorTest):
 * kinds[i] = 0 add(values[i]) -> 1/0, 1 contains(values[i]) -> 1/0, 2 size() -> count, 3 clear() -> 0. */
int32_t swim_kat_collector(const uint8_t* kinds, const int64_t* values, uint32_t n, int64_t* results);

#ifdef __cplusplus
}
#endif
#endif /* SWIM_H */
